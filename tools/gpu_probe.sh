# vq fix: reuse probe (default build), scale probe, then the LDS-poisoned build through the parity suite
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/p
L=assistive-vr-gym_amd/avr
timeout -k 10 300 python3 tools/b4_reuse.py > gpurun_out/p/reuse2.log 2>&1 || { rc=$?; echo rc=$rc; exit $rc; }
grep -v amdgpu gpurun_out/p/reuse2.log | tail -8 | cut -c1-200
timeout -k 10 300 env PROBE_SHORT=1 AVR_LIB=$L/libavr_poison.so python3 tools/b4_probe.py > gpurun_out/p/poison_probe.log 2>&1 || { rc=$?; echo rc=$rc; exit $rc; }
grep -v amdgpu gpurun_out/p/poison_probe.log | tail -3 | cut -c1-200
timeout -k 10 500 env AVR_LIB=$L/libavr_poison.so python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/p/poison_tests.log 2>&1
rc=$?
tail -3 gpurun_out/p/poison_tests.log
echo rc=$rc
