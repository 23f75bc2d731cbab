#!/bin/bash
# Round 6 gap decomposition: a traced bench run with its placements, a plain
# bench run, the regime replays + UMC calibration (tools/gap_decomp.py), the counter list, and
# the FETCH_SIZE / WRITE_SIZE calibration passes (tools/fetch_cal.py).
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/gpurun_out/${GAP_OUT:-r06_gap}
mkdir -p $O
GPUSCHED_BENCH_TRACE=$O/trace.json timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 \
  --dump-placements $O/place.json > $O/bench_traced.json 2> $O/bench_traced.err || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/bench_plain.json 2> $O/bench_plain.err || exit $?
timeout -k 10 500 python3 -u tools/gap_decomp.py --placements $O/place.json --out $O/decomp.json > $O/decomp.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_avail.txt 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/fc/p_$c -o run -- python3 $R/tools/fetch_cal.py $O/fc \
    > $O/fc_$c.log 2>&1 || exit $?
done
echo done
