#!/bin/bash
# Round 5: HBM copy-kernel probe (the bench's measured peak), and PMC (SQ + LDS passes) of k_replay on the fixed replay
# workload at 8 waves per SIMD (in-tree) and at 4 (W4: LDS slice padded) -- the occupancy end points of the
# two-envs-per-wave question (DESIGN §4 "k_replay, round 5").
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 build/tools/copy_probe > gpurun_out/r05b_copy_probe.txt 2>&1 || { cat gpurun_out/r05b_copy_probe.txt; exit 1; }
cat gpurun_out/r05b_copy_probe.txt
for v in base W4; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc_r05rp_${v}_sq -o run --output-format csv -- python3 tools/replay_bench.py --reps 2 > gpurun_out/pmc_r05rp_${v}_sq.log 2>&1 || { tail -5 gpurun_out/pmc_r05rp_${v}_sq.log; exit 1; }
  MFG_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_r05rp_${v}_lds -o run --output-format csv -- python3 tools/replay_bench.py --reps 2 > gpurun_out/pmc_r05rp_${v}_lds.log 2>&1 || { tail -5 gpurun_out/pmc_r05rp_${v}_lds.log; exit 1; }
  echo pmc $v ok
done
