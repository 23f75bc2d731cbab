#!/bin/bash
# HBM traffic of the stream-triad variants (PMC FETCH_SIZE/WRITE_SIZE in their own runs).
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_triad
cd /tmp && export TMPDIR=/tmp
for v in 1 3; do
  for n in 16777216 67108864; do
    timeout -k 10 120 python3 $R/tools/triad_one.py $n $v 20 >> $R/gpurun_out/pmc_triad/rates.txt 2>&1 || exit $?
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_triad/v${v}_n${n}_$c -o run -- python3 $R/tools/triad_one.py $n $v 20 > $R/gpurun_out/pmc_triad/v${v}_n${n}_$c.log 2>&1 || exit $?
    done
  done
done
cat $R/gpurun_out/pmc_triad/rates.txt
