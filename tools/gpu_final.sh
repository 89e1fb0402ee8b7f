# Final-tree profiles, then the round evidence with the fresh PMC summaries in place.
set -o pipefail
cd /root/repo
R=${ROUND:-r04}
bash tools/gpu_profile_all.sh || exit 21
cp gpurun_out/psum_$R/pmc_traffic.json gpurun_out/psum_${R}_scratch/pmc_scratch.json gpurun_out/psum_${R}_bedbath/pmc_bedbath.json profiles/ || exit 22
cp gpurun_out/psum_${R}_dressing/pmc_dressing.json profiles/ 2>/dev/null
bash tools/gpu_round.sh || exit 23
