# Round 5: where one lone 1024-env group's sub-step chain spends its time (the 4-group step is that
# chain + ~10 %): kernel trace of a 1024-env bench (one env group), the per-wave timeline of kernels
# a and B at 1024 and 4096 envs (AVR_WAVETIME build), and part B's SQ instruction / wait mix.
# Output: gpurun_out/r5prof/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5prof
O=gpurun_out/r5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt1k -o kt -- python3 bench.py --envs 1024 --steps 20 --warmup 3 --no-cpu-baseline --other-steps 0 > $O/kt1k.log 2>&1 || exit 11
timeout -k 10 200 python3 tools/wavetime.py 1024 > $O/wt1k.log 2>&1 || exit 12
timeout -k 10 200 python3 tools/wavetime.py 4096 > $O/wt4k.log 2>&1 || exit 13
AVR_GRAPH=0 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/sq -o sq -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-steps 0 > $O/sq.log 2>&1 || exit 14
find $O/kt1k -name '*stats*' -exec cp {} $O/ \;
mkdir -p $O/p && mv $O/sq $O/p/sq && AVR_PROF_OUT=$O python3 tools/rocpd_summary.py $O/p r5sq 4096 FeedingJaco-v0 > $O/sq_summary.txt 2>&1
rm -rf $O/p
rm -rf $O/kt1k
