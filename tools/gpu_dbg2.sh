set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/d2
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/d2/pt.log 2>&1
timeout -k 10 200 env AVR_LIB=assistive-vr-gym_amd/avr/libavr_base.so python3 tools/gpu_quick.py 8 3 > gpurun_out/d2/gq_base.log 2>&1
grep -E "passed|failed|Error|assert" gpurun_out/d2/pt.log | head -20
grep -E "settle:|worst" gpurun_out/d2/gq_base.log
