set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_margins.py tests/test_gpu_c3_full.py "tests/test_gpu_admm.py::test_admm_c5_full_batch" > gpurun_out/r4_t1.log 2>&1 || { tail -40 gpurun_out/r4_t1.log; exit 1; }
tail -3 gpurun_out/r4_t1.log
bash scripts/gpu_ab.sh base new1
