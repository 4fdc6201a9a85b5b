# C++ GPU data path: tests, then the b256 throughput of --device-data against the synthetic-batch
# --bench on the same box (a 10k-image synthetic Tiny-ImageNet JPEG directory)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cpp_data.py tests/test_cpp_dp.py -m gpu > gpurun_out/t_data.log 2>&1 || { echo "tests failed"; exit 1; }
echo "tests ok"
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'benchmarks')
from loader_bench import make_dataset
make_dataset('/tmp/tin10k', classes=100, per_class=100, val_per_class=2)
" || exit 1
for i in 1 2; do
timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | tail -1 > gpurun_out/data_syn_$i.json || exit 1
timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --data /tmp/tin10k --device-data --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce > gpurun_out/data_dev_$i.log 2>&1 || exit 1
tail -1 gpurun_out/data_dev_$i.log > gpurun_out/data_dev_$i.json
done
cat gpurun_out/data_syn_*.json gpurun_out/data_dev_*.json
