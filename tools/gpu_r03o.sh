#!/bin/bash
# A2C loop: engine-projection learner forward (test + profile), gather forward and rocBLAS for comparison.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_marl.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03o.log 2>&1 || { tail -30 gpurun_out/t_r03o.log; exit 1; }
tail -1 gpurun_out/t_r03o.log
for v in "" "--gather" "--blas cublas"; do
  timeout -k 10 300 python tools/prof_a2c.py $v > gpurun_out/prof_a2c.txt 2>&1 || { tail -20 gpurun_out/prof_a2c.txt; exit 1; }
  echo "== $v"; grep "^wall" gpurun_out/prof_a2c.txt
done
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/marl_r03o.json 2>gpurun_out/marl_r03o.err || { tail gpurun_out/marl_r03o.err; exit 1; }
cat gpurun_out/marl_r03o.json
