#!/bin/bash
# Adam + bf16-mirror kernel grid cap (PMLP_ADAM_BLOCKS): kernel-trace stats of the eager
# optimizer-step probe, two interleaved rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/adam_ab
mkdir -p $O
for r in 1 2; do
  for b in ${ADAM_AB_BLOCKS:-1024 512 256}; do
    PMLP_ADAM_BLOCKS=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/b$b -o run --output-format csv \
        -- python tools/probes/update_step_time.py > $O/b$b.log 2>&1 || exit 3
    echo "== PMLP_ADAM_BLOCKS=$b round $r"; python tools/kernel_stats_top.py $O/b$b 40 | grep -E "k_adam"
    rm -rf $O/b$b
  done
done
