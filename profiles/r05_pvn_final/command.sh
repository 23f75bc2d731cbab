#!/bin/bash
OUT_NAME=r05_pvn_final SEEDS="0 1 2" POLICIES="greedy planner planner-e1 planner-e2" bash tools/archive/gpu_r05_pvn.sh
