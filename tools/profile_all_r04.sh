# Every bench config's committed profile at the current tree (tools/profile_r04.sh).
set -o pipefail
cd "$(dirname "$0")/.."
for c in "S2" "S1" "S4" "S4 20000" "S2shard 8" "S2shard 4" "region 128"; do
  bash tools/profile_r04.sh $c > /dev/null 2>&1 || { echo "profile $c failed"; exit 1; }
  n=$(echo $c | tr ' ' '_'); [ "$c" = "region 128" ] && n=region_415x128
  [ "${c%% *}" = S2shard ] && n=S2shard_${c##* }
  echo "$c: $(tail -1 gpurun_out/prof4_$n/summary.log | cut -c1-400)"
done
