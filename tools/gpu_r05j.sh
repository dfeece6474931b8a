#!/bin/bash
# Round 5: A2C learner device time per phase (bench settings, cap 32).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_a2c_phases.py > gpurun_out/r05j_a2c_phases.json 2> gpurun_out/r05j_a2c_phases.err || { tail -10 gpurun_out/r05j_a2c_phases.err; exit 1; }
cat gpurun_out/r05j_a2c_phases.json
timeout -k 10 300 python tools/prof_a2c.py > gpurun_out/r05j_prof_a2c.txt 2>&1 || { tail -10 gpurun_out/r05j_prof_a2c.txt; exit 1; }
head -40 gpurun_out/r05j_prof_a2c.txt
