#!/bin/bash
# Split-K slab combine: slab groups per element quad (default) vs one thread per quad
# (PMLP_REDUCE_GROUPS=0); fused-update parity tests first, then kernel-trace stats of the
# eager optimizer-step probe, two interleaved rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/reduce_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_recurrent.py -x -q --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for g in ${REDUCE_AB:-1 0}; do
    PMLP_REDUCE_GROUPS=${g%%:*} PMLP_REDUCE_SPT=${g##*:} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/g$g -o run --output-format csv \
        -- python tools/probes/update_step_time.py > $O/g$g.log 2>&1 || exit 3
    echo "== PMLP_REDUCE_GROUPS=$g round $r"; python tools/kernel_stats_top.py $O/g$g 40 | grep -E "k_reduce_jobs"
    rm -rf $O/g$g
  done
done
