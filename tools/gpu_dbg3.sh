cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/d3
timeout -k 10 200 python3 tools/dbg3.py 100 > gpurun_out/d3/new.log 2>&1

grep -v amdgpu gpurun_out/d3/new.log | cut -c1-200


