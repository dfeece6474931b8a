cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MFG_HIP_LIB=build/ablate/libmfg_hip_OLD.so timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_facade.py -k rooms4 > gpurun_out/r04j_old.txt 2>&1; tail -3 gpurun_out/r04j_old.txt
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_facade.py tests/test_gpu_parity.py -k "rooms4 or alltest16" > gpurun_out/r04j_new.txt 2>&1; tail -8 gpurun_out/r04j_new.txt
