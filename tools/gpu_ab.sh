# A/B exactness (base lib vs current lib, final states after settle + steps), GPU tests, bench
# kernel-trace split.  Usage: bash tools/gpu_ab.sh [pytest-args]
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
L=assistive-vr-gym_amd/avr
timeout -k 10 200 env AVR_LIB=$L/libavr_base.so python3 tools/ab_state.py gpurun_out/ab/base.npy 512 5 > gpurun_out/ab/base.log 2>&1 && \
timeout -k 10 200 python3 tools/ab_state.py gpurun_out/ab/new.npy 512 5 > gpurun_out/ab/new.log 2>&1 && \
python3 -c "
import numpy as np
a=np.load('gpurun_out/ab/base.npy'); b=np.load('gpurun_out/ab/new.npy')
d=np.abs(a-b); print('A/B: identical envs %d/%d, max|diff| %.3g' % ((d.max(1)==0).sum(), len(a), d.max()))
" && \
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/kt_bench.log 2>&1
rc=$?
tail -3 gpurun_out/ab/pytest_gpu.log
grep '"value"' gpurun_out/ab/kt_bench.log | cut -c1-200
find gpurun_out/ab/kt -name "*stats.csv" | head -3 | xargs -r cat | cut -d, -f1-5 | head -8
echo rc=$rc
