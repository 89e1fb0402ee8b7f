# Round profile (PMC passes with direct launches, AVR_GRAPH=0: the counters are per dispatch and the
# kernels are the same; the kernel traces and the bench line use the default graph replay): rocprofv3 kernel-trace stats of the default bench workload, then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix), then the full bench line (with the CPU
# baseline).  Summaries: python tools/rocpd_summary.py gpurun_out/prof <tag>.
# The rocpd databases go to /tmp/prof (they outgrow gpurun_out's 64 MiB); only the summaries and
# logs land under gpurun_out/.  The profiled runs time the task alone (--other-steps 0,
# --sync-steps 0); bench.py's progress lines on stderr keep the logs growing.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/prof /tmp/prof
TASK=${TASK:-FeedingJaco-v0}
B="bench.py --task $TASK --steps 20 --warmup 3 --no-cpu-baseline --other-steps 0 --sync-steps 0"
B5="bench.py --task $TASK --steps 20 --warmup 5 --no-cpu-baseline --other-steps 0 --sync-steps 0"
(rocm-smi --showclocks --showuse --showpower 2>&1 || true) > gpurun_out/prof/smi_before.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof/kt -o kt -- python3 $B > gpurun_out/prof/kt_bench.log 2>&1 && \
AVR_ENV_GROUPS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof/kt1 -o kt1 -- python3 $B > gpurun_out/prof/kt1_bench.log 2>&1 && \
AVR_GRAPH=0 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d /tmp/prof/fetch -o fetch -- python3 $B5 > gpurun_out/prof/fetch.log 2>&1 && \
AVR_GRAPH=0 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d /tmp/prof/write -o write -- python3 $B5 > gpurun_out/prof/write.log 2>&1 && \
AVR_GRAPH=0 timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d /tmp/prof/sq -o sq -- python3 $B5 > gpurun_out/prof/sq.log 2>&1 && \
timeout -k 10 600 python3 bench.py --task $TASK --other-steps 0 > gpurun_out/prof/bench_full.log 2>&1
rc=$?
(rocm-smi --showclocks --showuse --showpower 2>&1 || true) > gpurun_out/prof/smi_after.txt
# summaries on the box (the rocpd databases are too large to copy back), then drop the databases
PS=gpurun_out/psum_${TAG:-r03}; mkdir -p $PS && AVR_PROF_OUT=$PS python3 tools/rocpd_summary.py /tmp/prof ${TAG:-r03} ${ENVS:-4096} $TASK > $PS/summary.txt 2>&1
cp gpurun_out/prof/*.txt gpurun_out/prof/*.log $PS/ 2>/dev/null
rm -rf gpurun_out/prof /tmp/prof
tail -1 $PS/bench_full.log | cut -c1-600
head -24 $PS/summary.txt
echo rc=$rc
exit $rc
