mkdir -p gpurun_out/s3a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3a/gpu_tests.log 2>&1 && tail -2 gpurun_out/s3a/gpu_tests.log &&
timeout -k 10 400 python bench.py > gpurun_out/s3a/bench.log 2>&1 && tail -1 gpurun_out/s3a/bench.log | cut -c1-400 &&
for sg in 0 32768; do DHTGPU_F2SEG=$sg timeout -k 10 120 python tools/batch_probe.py --reps 500 --inflight 2 > gpurun_out/s3a/probe_seg$sg.log 2>&1 || exit 1; DHTGPU_F2SEG=$sg DHTGPU_DBG=256 timeout -k 10 120 python tools/batch_probe.py --reps 1 > gpurun_out/s3a/stamps_seg$sg.log 2>&1 || exit 1; grep -h "ms/call\|phases" gpurun_out/s3a/probe_seg$sg.log; done
