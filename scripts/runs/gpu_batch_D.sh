cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "batch" > gpurun_out/pytest_gpu_b2.log 2>&1 && tail -3 gpurun_out/pytest_gpu_b2.log && \
timeout -k 10 300 python bench.py --workload D --scenes 1 --steps 3 --warmup 1 > gpurun_out/bench_D_b2.log 2>&1 && tail -1 gpurun_out/bench_D_b2.log | cut -c1-250 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profD_b2 -o kt --output-format csv -- python bench.py --workload D --scenes 1 --steps 1 --warmup 1 > gpurun_out/profD_b2.log 2>&1 && echo done
