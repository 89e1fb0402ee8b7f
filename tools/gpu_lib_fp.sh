# Bit-identity of the working tree's libavr.so against an experiment library of the same tree
# (OLD_LIB, loaded through AVR_LIB): tools/fingerprint.py on the three rigid tasks; then TESTS.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/fp
for t in ${FP_TASKS:-0 1 2}; do
  FP_STATES=gpurun_out/fp/S$t.npz TASK=$t AVR_LIB=$OLD_LIB timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/fp/old$t.npz > gpurun_out/fp/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/fp/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/fp/new$t.npz gpurun_out/fp/old$t.npz > gpurun_out/fp/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/fp/new$t.log
done
rm -f gpurun_out/fp/*.npz
[ -n "$TESTS" ] || exit 0
timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread $TESTS > gpurun_out/fp_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fp_tests.log; exit $rc
