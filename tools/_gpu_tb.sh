mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk16.py tests/test_gpu_retrieval.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1; rc=$?; tail -5 gpurun_out/t16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/microbench_topk.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/mb_topk.log
