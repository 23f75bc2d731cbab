#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 90 python3 -u tools/smi_proc_probe.py > gpurun_out/smi_proc_probe.log 2>&1 || exit $?
echo done
