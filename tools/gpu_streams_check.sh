set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "streams" > gpurun_out/pt_streams.log 2>&1 || { tail -30 gpurun_out/pt_streams.log; exit 1; }
tail -2 gpurun_out/pt_streams.log
./tools/gpu_streams.sh
