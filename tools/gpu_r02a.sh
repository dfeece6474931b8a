set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_timed_path.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -15 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -5 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 400 --warmup 600 > gpurun_out/b1.json 2> gpurun_out/b1.err; rc=$?; cat gpurun_out/b1.json; tail -3 gpurun_out/b1.err; exit $rc
