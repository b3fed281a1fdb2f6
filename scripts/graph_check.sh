cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "captured or mirror" > gpurun_out/pytest_graph.log 2>&1; echo "pytest rc=$?" >> gpurun_out/graph_status.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph > gpurun_out/bench_graph.log 2>&1; echo "bench graph rc=$?" >> gpurun_out/graph_status.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --arch resnet18 --image-size 32 --num-classes 10 > gpurun_out/bench_r18.log 2>&1; echo "r18 rc=$?" >> gpurun_out/graph_status.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --arch resnet18 --image-size 32 --num-classes 10 --graph > gpurun_out/bench_r18_graph.log 2>&1; echo "r18 graph rc=$?" >> gpurun_out/graph_status.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --arch resnet18 --image-size 32 --num-classes 10 --impl torch > gpurun_out/bench_r18_torch.log 2>&1; echo "r18 torch rc=$?" >> gpurun_out/graph_status.txt
