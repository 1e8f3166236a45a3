#!/bin/bash
# Profiles of the bench command for profiles/ (run on the GPU box; tools/collect_profiles.sh
# copies the summaries into profiles/ with the round's prefix):
#   1. rocprofv3 --kernel-trace --stats of a short bench run (no CPU legs, every line);
#   2. PMC FETCH_SIZE / WRITE_SIZE passes (tools/pmc_bench.sh);
#   3. SQ counter passes (tools/pmc_sq_bench.sh);
#   4. the C5 (dense MFMA) passes (tools/pmc_concat.sh), merged into 2.'s traffic file.
# Each summary carries the sha256 of the library it measured (bench.py uses only a matching one).
# Each step has its own time limit; the script stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- python bench.py --cpu-seconds 0 --bp-ebn0-extra --steps 10 --warmup 2 --detail-dir $O > $O/bench.json 2> $O/bench.err
bash tools/pmc_bench.sh
bash tools/pmc_sq_bench.sh
bash tools/pmc_concat.sh
python tools/pmc_concat.py gpurun_out/pmcc gpurun_out/pmcb/traffic.json > gpurun_out/pmcc/summary.json
echo prof_round done
