cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/sweep_ws2.txt; : > $O
for E in "X=0" "DCNN_WGRAD_STREAM=1"; do
  for cfg in "--model resnet50_tiny_imagenet --batch 32" "--batch 64" "--batch 128" "--batch 256"; do
    env $E timeout -k 10 240 python bench.py --steps 30 --warmup 5 $cfg > gpurun_out/cur.out 2>&1 || exit $?
    echo "$E $cfg :: $(grep '^{' gpurun_out/cur.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O
  done
done
cat $O
