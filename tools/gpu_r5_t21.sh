# Round 5: narrowphase results without the point for pairs without contact -- the parity and
# bit-identity tests that cover the narrowphase hand-over, then the FeedingJaco profile
# (tools/gpu_profile.sh; summaries in gpurun_out/psum_r05/).  Output: gpurun_out/r5t21/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t21
timeout -k 10 600 python3 -u -m pytest -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_narrowphase_pairs.py -k "golden or bit_identical or one_substep or narrowphase or rollout or poison" > gpurun_out/r5t21/tests.log 2>&1
rc=$?; echo tests rc=$rc; case $rc in 0) ;; *) exit $rc ;; esac
TASK=FeedingJaco-v0 TAG=r05 bash tools/gpu_profile.sh > gpurun_out/prof_feeding.log 2>&1 || exit 11
