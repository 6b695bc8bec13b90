set -o pipefail
O=gpurun_out/r06_s1; mkdir -p $O
{ cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpuset.cpus.effective 2>&1; nproc; python -c "import os;print(len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:40])"; lscpu | head -20; } > $O/host.txt 2>&1
timeout -k 10 300 python -u tools/rxq_lifecycle_probe.py --mode owned --cycles 16 > $O/probe_owned.log 2>&1 &&
timeout -k 10 200 python -u tools/rxq_lifecycle_probe.py --mode raw --cycles 40 > $O/probe_raw.log 2>&1 &&
timeout -k 10 400 python -u tools/rxq_lifecycle_probe.py --mode registered --cycles 40 > $O/probe_registered.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pdsch_tail_gpu.py tests/test_tail_stream_gpu.py tests/test_rx_queue_gpu.py > $O/pytest.log 2>&1
