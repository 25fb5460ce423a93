#!/bin/bash
# Split-K target (PMLP_KSPLIT_TARGET workgroups per weight-gradient job) with the slab-group
# combine: eager per-group times of one optimizer step, two interleaved rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for t in 128 256 64; do
    echo "== PMLP_KSPLIT_TARGET=$t round $r"
    PMLP_KSPLIT_TARGET=$t timeout -k 10 200 python tools/probes/update_step_time.py > gpurun_out/ks_$t.log 2>&1 || exit 3
    grep -E "PART_TN|reduce|TOTAL" gpurun_out/ks_$t.log
  done
done
