#!/bin/bash
# Round 5: the two-wave replay with the MT state in the producer's registers. Parity first (grid128 fixtures and
# batched C5 envs take it by occupancy; C2-C4 and the B = 65,536 timed-path tests with it forced, -DMFG_REPLAY2=2),
# then C5 throughput.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05g
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "grid128_64" > gpurun_out/${T}_c5_tests.txt 2>&1 \
  || { tail -40 gpurun_out/${T}_c5_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_c5_tests.txt
MFG_HIP_LIB=build/ablate/libmfg_hip_RP2F.so timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timed_path.py -k "large8 or rooms4 or alltest16 or timed_path_k8 or maint_rooms or table_path or full_temper" > gpurun_out/${T}_rp2f_tests.txt 2>&1 \
  || { tail -40 gpurun_out/${T}_rp2f_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_rp2f_tests.txt
timeout -k 10 500 python bench.py --no-cpu-baseline --config grid128_64.yaml --batch 131072 --fuse 1 --steps 10 --warmup 3 --alt-steps 0 --packed-steps 0 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { tail -5 gpurun_out/${T}_c5.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], {k:v.get('mean_launch_ms') for k,v in d['roofline']['kernels'].items() if isinstance(v,dict)})" gpurun_out/${T}_c5.json
