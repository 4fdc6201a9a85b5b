# the round-end check: full GPU suite, smoke, headline bench
cd $GRAFT_REPO_ROOT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/t_full.log 2>&1
rc=$?
tail -5 gpurun_out/t_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || exit 1
tail -1 gpurun_out/bench_full.log
