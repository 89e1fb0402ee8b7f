set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
AVR_ENV_GROUPS=1 timeout -k 10 200 python3 tools/wavetime.py 4096 > gpurun_out/wt.log 2>&1 && \
AVR_ENV_GROUPS=1 timeout -k 10 200 python3 tools/wavetime.py 1024 > gpurun_out/wt1k.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/wt.log | tail -12
grep -v amdgpu.ids gpurun_out/wt1k.log | tail -12
echo rc=$rc
