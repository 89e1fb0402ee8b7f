# Round 5 diagnostics: the dressing parity tests and smoke after the qnlerp rounding fix, the PR2
# launch-shape test with contact picks and the fp32 rounding ensemble, and the sub-step divergence
# of the ScratchItch contact pool state 31 and of the FeedingJaco arm-in-wheelchair state (EPA
# budget off).  A test failure does not stop the script; a fault, abort or time limit does.
# Output: gpurun_out/r5d/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5d
run() {   # run <log> <seconds> <command...>
    local log=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > gpurun_out/r5d/$log 2>&1
    local rc=$?
    echo "$log rc=$rc"
    case $rc in 124|134|137|139) exit $rc ;; esac
    return 0
}
run dress.log 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_dressing.py
run smoke.log 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run launch.log 600 python3 -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu tests/test_pr2_launch_shape.py -k launch_shape
TASK=1 K=31 STEPS=3 run sub_s31.log 240 python3 -u tools/dbg_substeps.py
TASK=0 STEPS=4 run sub_wheel.log 240 python3 -u tools/dbg_substeps.py
