set -o pipefail
mkdir -p gpurun_out
bash tools/profile_round.sh r02 S2 || exit 1
bash tools/profile_round.sh r02 S1 || exit 1
ls gpurun_out/prof_r02_S2/trace
