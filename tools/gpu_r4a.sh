# Round-4 check: FeedingJaco bit-identity of the working tree against a previous build (AB_ROOT, default _ab2/: a
# git worktree of the previous commit with its libavr.so built beforehand); the PR2 tasks'
# fingerprints (torsional friction changes them: reported, not required equal); then the GPU tests
# this round touched.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
for t in ${FP_TASKS:-0 1 2}; do
  FP_STATES=gpurun_out/ab/S$t.npz TASK=$t AVR_FP_ROOT=${AB_ROOT:-/root/repo/_ab2} timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/ab/old$t.npz > gpurun_out/ab/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/ab/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/ab/new$t.npz gpurun_out/ab/old$t.npz > gpurun_out/ab/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/ab/new$t.log
done
[ -n "$KEEP_NPZ" ] || rm -f gpurun_out/ab/*.npz
[ -n "$TESTS" ] || exit 0
timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread $TESTS > gpurun_out/r4_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_tests.log; exit $rc
