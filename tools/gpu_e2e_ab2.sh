set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_stream.py tests/test_inflate.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/stream_gpu_tests.log 2>&1 || { tail -20 gpurun_out/stream_gpu_tests.log; exit 1; }
tail -1 gpurun_out/stream_gpu_tests.log
E2E_BASE_INFLATE=0 E2E_INFLATE_AB=1 timeout -k 10 700 bash tools/gpu_e2e_chrom.sh 3 > gpurun_out/e2e_chrom.log 2>&1 || exit 1
echo done
