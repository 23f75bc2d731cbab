#!/bin/bash
# pipelined virtual node with alternative level-1 tables (tools/pipelined_vn.py POLICY_ENV)
OUT_NAME=r05_pvn_levels POLICIES="greedy planner planner-e1old planner-e1c planner-e1a" bash tools/archive/gpu_r05_pvn.sh
