cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_gap2; mkdir -p $O
timeout -k 10 200 python3 -u tools/gap_decomp.py --placements tools/inputs/r06_place_seed0.json --only replay,replay_la2,replay_nograph --mask-units "" --skip-cal --reps 3 --out $O/q32.json > $O/q32.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python3 -u tools/gap_decomp.py --placements tools/inputs/r06_place_seed0.json --only replay,replay_la2,replay_nograph --mask-units "" --skip-cal --reps 3 --out $O/q16.json > $O/q16.log 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 -u tools/gap_decomp.py --placements tools/inputs/r06_place_seed0.json --only replay,replay_la2 --mask-units "" --skip-cal --reps 3 --out $O/q8.json > $O/q8.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
echo done
