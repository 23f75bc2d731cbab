#!/bin/bash
# Round 5: per-pod kernel policy A/B (20-step bench, interleaved): off vs risk.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python tools/ab.py --rounds 4 --steps 20 --warmup 5 --out gpurun_out/r05_policy_ab \
  --arm off="--kernel-policy off" --arm risk="--kernel-policy risk"
