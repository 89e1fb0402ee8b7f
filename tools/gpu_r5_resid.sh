# Round 5: the PGS residual-threshold build -- GPU suite, smoke, contact-pool diagnostics and the
# four bench lines.  A test failure does not stop the script; a fault, abort or time limit does.
# Output: gpurun_out/r5r/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5r
run() {   # run <log> <seconds> <command...>
    local log=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > gpurun_out/r5r/$log 2>&1
    local rc=$?
    echo "$log rc=$rc"
    case $rc in 124|134|137|139) exit $rc ;; esac
    return 0
}
TASK=0 run pool_wheel.log 200 python3 -u tools/dbg_pool_diff.py
TASK=1 K=27 run pool_s27.log 200 python3 -u tools/dbg_pool_diff.py
TASK=1 K=27 SA=50 SB=165 run np27.log 300 python3 -u tools/dbg_np_state.py
run pytest.log 800 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run smoke.log 300 python3 -c "import __graft_entry__ as g; g.smoke()"
for T in FeedingJaco-v0 ScratchItchPR2-v0 BedBathingPR2-v0; do
  run bench_$T.json 200 python3 bench.py --task $T --steps 20 --warmup 5 --no-cpu-baseline --other-steps 0
done
