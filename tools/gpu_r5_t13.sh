# Round 5: double simplex solve only (fp32 GJK state), tetra faces lane-parallel; stalls above 0.1 mm rerun;
# FeedingJaco / ScratchItch benches against the previous build (_ab/libavr_head.so).
# Output: gpurun_out/r5t13/, gpurun_out/ab/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t13
run() {   # run <log> <seconds> <command...>
    local log=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > gpurun_out/r5t13/$log 2>&1
    local rc=$?
    echo "$log rc=$rc"
    case $rc in 124|134|137|139) exit $rc ;; esac
    return 0
}
TASK=1 K=27 SA=50 SB=165 run np27.log 300 python3 -u tools/dbg_np_state.py
run tests.log 700 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_narrowphase_pairs.py tests/test_pr2_launch_shape.py "tests/test_gpu_parity.py::test_coop_capped_env_drift_vs_oracle"
VARIANTS="default head" ROUNDS=2 bash tools/gpu_ab_variants.sh > gpurun_out/r5t13/ab.log 2>&1 || exit 22
TASK=ScratchItchPR2-v0 VARIANTS="default head" ROUNDS=1 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t13/ab.log 2>&1 || exit 23
TASK=BedBathingPR2-v0 VARIANTS="default head" ROUNDS=1 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t13/ab.log 2>&1 || exit 24
