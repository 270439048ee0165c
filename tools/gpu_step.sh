set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in on off; do
HC_PHMM_CHAIN=$c timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_chain_$c -o run -- python3 tools/sweep.py S1w:1000000 --runs 2 > gpurun_out/pmc_chain_$c.log 2>&1 || exit 1
done
echo ok
