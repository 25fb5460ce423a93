#!/bin/bash
# Round 6: the PGS sweep-count A/B on one box -- k_step vs sweeps (Go2 4096, H1_2 8192), and the
# Go2 300-iteration learning curve at the chosen 5 sweeps and at the former 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-r6_sweeps}
mkdir -p $O
timeout -k 10 300 python tools/probes/sweeps_ab.py go2 4096 3 8 5 6 4 > $O/kstep_go2.txt 2>&1 || exit 2
timeout -k 10 300 python tools/probes/sweeps_ab.py h1_2 8192 2 8 6 5 > $O/kstep_h1_2.txt 2>&1 || exit 3
timeout -k 10 300 python tools/learn_curve.py go2 300 4096 - 5 > $O/learn_go2_5.log 2>&1 || exit 4
timeout -k 10 300 python tools/learn_curve.py go2 300 4096 - 8 > $O/learn_go2_8.log 2>&1 || exit 5
grep -h "k_step" $O/kstep_*.txt
for f in $O/learn_go2_*.log; do tail -n 2 $f; done
