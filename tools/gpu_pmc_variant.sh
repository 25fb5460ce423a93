# time + FETCH/WRITE for one library build: bash tools/gpu_pmc_variant.sh <lib.so> <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export LEGGEDSIM_LIB=$1
T=$2
mkdir -p gpurun_out
rm -rf gpurun_out/pt_$T gpurun_out/pf_$T gpurun_out/pw_$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pt_$T -o run --output-format csv -- python tools/profile_env.py go2 4096 60 > /dev/null 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf_$T -o run --output-format csv -- python tools/profile_env.py go2 4096 20 > /dev/null 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pw_$T -o run --output-format csv -- python tools/profile_env.py go2 4096 20 > /dev/null 2>&1 || exit 4
python tools/pmc_summary.py gpurun_out/pt_$T gpurun_out/pf_$T gpurun_out/pw_$T k_step gpurun_out/pmc_$T.json
