# Round 5: narrowphase near contact (queries 1 mm from contact) against the fp64 restatement.
# Output: gpurun_out/r5t26/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t26
timeout -k 10 300 python3 -u -m pytest tests/test_narrowphase_pairs.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t26/np.log 2>&1; echo "np tests rc=$?"
grep -E "misses|passed|failed|Error" gpurun_out/r5t26/np.log
