# Round 4, step 13: every bench config's committed profile at the tree, then
# the closing check (GPU suite, smoke, default bench line).
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/profile_all_r04.sh || exit 1
bash tools/gpu_r4_final.sh
