set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for lib in new old; do
  if [ $lib = old ]; then export HC_PHMM_LIB=build_ab/libold.so; else unset HC_PHMM_LIB; fi
  echo -n "$lib "; timeout -k 10 300 python -u tools/e2e_ab.py 2>> gpurun_out/e2e_ab.err || exit 1
done
done
