# Round 5: instruction-fetch counters per kernel (FeedingJaco bench, direct launches): SQC
# instruction-cache requests / hits / misses and the wave-cycles spent waiting for an instruction.
# Summary: gpurun_out/r5ic/summary.txt
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ic
AVR_GRAPH=0 timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_BUSY_CYCLES -d gpurun_out/r5ic/db -o ic -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-steps 0 > gpurun_out/r5ic/run.log 2>&1
rc=$?; echo pmc rc=$rc
python3 tools/pmc_counters_summary.py gpurun_out/r5ic/db SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_BUSY_CYCLES > gpurun_out/r5ic/summary.txt 2>&1
echo summary rc=$?

rm -rf gpurun_out/r5ic/db
exit $rc
