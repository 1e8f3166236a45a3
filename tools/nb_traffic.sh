#!/bin/bash
# Notebook / C4 engine check: their GPU tests, then the PMC traffic passes of
# tools/pmc_bench.sh (FETCH_SIZE / WRITE_SIZE over a short bench run).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nbt
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread "tests/test_amp_gpu.py::test_notebook_block2_vs_general_engine" "tests/test_amp_gpu.py::test_notebook_geometry_vs_oracle" "tests/test_amp_gpu.py::test_c4_block_engine_vs_general_engine" "tests/test_amp_gpu.py::test_c4_block_engine_vs_oracle" > gpurun_out/nbt/tests.log 2>&1
bash tools/pmc_bench.sh
