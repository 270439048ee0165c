# Round-3 committed profiles of the bench configs at the current HEAD (warm
# kernel traces + PMC passes), one config after another; stops at the first failure.
set -o pipefail
bash tools/profile_r03.sh S2 > gpurun_out/prof3_S2.log 2>&1 || { echo "S2 failed"; exit 1; }
bash tools/profile_r03.sh S1 > gpurun_out/prof3_S1.log 2>&1 || { echo "S1 failed"; exit 1; }
bash tools/profile_r03.sh S4 > gpurun_out/prof3_S4.log 2>&1 || { echo "S4 failed"; exit 1; }
bash tools/profile_r03.sh S4 20000 > gpurun_out/prof3_S4_20000.log 2>&1 || { echo "S4-20k failed"; exit 1; }
bash tools/profile_r03.sh region 128 > gpurun_out/prof3_region.log 2>&1 || { echo "region failed"; exit 1; }
