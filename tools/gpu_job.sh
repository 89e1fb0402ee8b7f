# Parameterised GPU-box job (replaces the one-off per-experiment scripts of earlier rounds).
#
#   bash tools/gpu_job.sh <outdir> <step> [<step> ...]
#
# Each <step> is "log:seconds:command" and runs from the repo root as
#   timeout -k 10 <seconds> <command> > gpurun_out/<outdir>/<log> 2>&1
# Steps run in order; a step that times out, aborts or segfaults (124/134/137/139) ends the job
# with its code, and nothing further touches the GPU.  Other non-zero codes are reported and the
# job goes on (a failing test file does not hide the benches after it); the job's exit code is the
# first such code.  Examples:
#   bash tools/gpu_job.sh r6a "tests.log:600:python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_scratch.py"
#   bash tools/gpu_job.sh r6b "b.json:200:python3 bench.py --steps 30 --no-cpu-baseline --other-steps 0"
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
out=gpurun_out/$1; shift
mkdir -p "$out"
first=0
for step in "$@"; do
    log=${step%%:*}; rest=${step#*:}
    secs=${rest%%:*}; cmd=${rest#*:}
    timeout -k 10 "$secs" bash -c "$cmd" > "$out/$log" 2>&1
    rc=$?
    echo "$log rc=$rc"
    tail -n 3 "$out/$log"
    case $rc in 124|134|137|139) exit $rc ;; esac
    if [ $rc -ne 0 ] && [ $first -eq 0 ]; then first=$rc; fi
done
exit $first
