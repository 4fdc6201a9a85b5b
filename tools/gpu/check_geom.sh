cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_cpp_geometry.py > gpurun_out/t_geom.log 2>&1
echo "geometry rc=$?"
bash tools/gpu/probe_pg.sh
