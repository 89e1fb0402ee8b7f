# Round 5: narrowphase near-contact tests including FeedingJaco's food spheres against the spoon
# and bowl hulls.  Output: gpurun_out/r5t29/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t29
timeout -k 10 300 python3 -u -m pytest tests/test_narrowphase_pairs.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t29/np.log 2>&1; echo "np tests rc=$?"
grep -E "misses|passed|failed" gpurun_out/r5t29/np.log
