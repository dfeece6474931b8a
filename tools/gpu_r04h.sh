#!/bin/bash
# Issue/branch/latency probe, then k_replay branch-count variants A/B on the fixed workload (exact: equal state sha).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./build/issue_probe > gpurun_out/r04h_issue_probe.txt 2>&1 || { tail -5 gpurun_out/r04h_issue_probe.txt; exit 1; }
cat gpurun_out/r04h_issue_probe.txt
bash tools/replay_ab.sh "$@"
