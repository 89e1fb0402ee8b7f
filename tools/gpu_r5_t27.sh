# Round 5: the cooperative fp32 GJK (big hulls, penetrating pairs) checks the duality gap on a
# no-progress stop and reruns a stall in double -- fingerprints against the previous build,
# near-contact narrowphase tests, interleaved benches, then the whole GPU suite.
# Output: gpurun_out/r5t27/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t27
for t in 0 1 2; do
  FP_STATES=gpurun_out/r5t27/S$t.npz TASK=$t AVR_LIB=/root/repo/_ab/libavr_prev.so timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t27/old$t.npz > gpurun_out/r5t27/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/r5t27/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t27/new$t.npz gpurun_out/r5t27/old$t.npz > gpurun_out/r5t27/new$t.log 2>&1; echo "task $t rc=$?"; tail -2 gpurun_out/r5t27/new$t.log
done
rm -f gpurun_out/r5t27/*.npz
timeout -k 10 300 python3 -u -m pytest tests/test_narrowphase_pairs.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t27/np.log 2>&1; echo "np tests rc=$?"
grep -E "misses|passed|failed" gpurun_out/r5t27/np.log
for T in FeedingJaco-v0 ScratchItchPR2-v0 BedBathingPR2-v0; do
  TASK=$T VARIANTS="default prev" ROUNDS=2 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t27/ab.log 2>&1 || exit 12
done
cat gpurun_out/r5t27/ab.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t27/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "FAILED|passed|failed" gpurun_out/r5t27/pytest.log | tail -5
