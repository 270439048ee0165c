# Every bench config's committed profile at the current tree (round 4).
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/profile_all_r04.sh
