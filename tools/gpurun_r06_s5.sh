set -o pipefail
# bench + profiles first (tools/r06_gpu.sh without tests), then the whole GPU suite
bash tools/r06_gpu.sh r06_s5 bench trace pmc c2pmc none &&
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s5/pytest.log 2>&1
