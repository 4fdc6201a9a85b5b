# A/B of environment knobs on the C++ headline step (same box, alternating runs): TAG then
# "NAME=VALUE" settings (one run set per setting, "-" = defaults); prints img/s and the final loss
TAG=$1; shift
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for cfg in "$@"; do
    if [ "$cfg" = "-" ]; then envs=""; else envs="$cfg"; fi
    v=$(env $envs timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch ${AB_BATCH:-256} --model ${AB_MODEL:-resnet18_tiny_imagenet} --steps 40 --warmup 8 --loss softmax_ce | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], repr(d['loss']))") || exit 1
    echo "$TAG rep$rep [$cfg] $v" | tee -a gpurun_out/ab_$TAG.txt
  done
done
