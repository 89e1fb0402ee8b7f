# Final-tree profiles, then the round evidence with the fresh PMC summaries in place.
set -o pipefail
cd /root/repo
bash tools/gpu_profile_all.sh || exit 21
cp gpurun_out/psum_r03/pmc_traffic.json gpurun_out/psum_r03_scratch/pmc_scratch.json gpurun_out/psum_r03_bedbath/pmc_bedbath.json profiles/ || exit 22
bash tools/gpu_round.sh || exit 23
