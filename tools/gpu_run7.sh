#!/bin/bash
# full GPU test suite (kernels, models, pipeline on cuda:0)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t7.log 2>&1
