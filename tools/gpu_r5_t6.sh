# Round 5: double-precision cooperative GJK (lane no-progress handed over) -- the narrowphase pair tests, the state-27 neighbourhood, the
# PR2 launch-shape tests, the wheelchair drift and a FeedingJaco bench.  Output: gpurun_out/r5t6/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t6
run() {   # run <log> <seconds> <command...>
    local log=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > gpurun_out/r5t6/$log 2>&1
    local rc=$?
    echo "$log rc=$rc"
    case $rc in 124|134|137|139) exit $rc ;; esac
    return 0
}
TASK=1 K=27 SA=50 SB=165 run np27.log 300 python3 -u tools/dbg_np_state.py
run tests.log 700 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_narrowphase_pairs.py tests/test_pr2_launch_shape.py -k "not contact_regime" "tests/test_gpu_parity.py::test_coop_capped_env_drift_vs_oracle"
run bench_feeding.json 200 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --other-steps 0
timeout -k 10 200 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/mb/chain.hip -o /tmp/avr_chain_mb > gpurun_out/r5t6/chain_build.log 2>&1 || exit 21
run chain.log 120 /tmp/avr_chain_mb
