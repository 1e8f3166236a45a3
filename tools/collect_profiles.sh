#!/bin/bash
# Copies the summaries of tools/prof_round.sh (gpurun_out/, merged back from the GPU box) into
# profiles/ with the prefix $1 (e.g. r04_final): kernel stats of the bench command, the PMC
# traffic file (with the C5 section and the library digest), the SQ summary.
set -e
cd "$(dirname "$0")/.."
p=${1:?prefix}
cp gpurun_out/prof/ks/run_kernel_stats.csv profiles/${p}_bench_kernel_stats.csv
cp gpurun_out/prof/bench.json profiles/${p}_prof_bench.json
for f in gpurun_out/prof/bench_detail_*.json; do [ -f "$f" ] && cp "$f" profiles/${p}_prof_$(basename $f); done
cp gpurun_out/pmcb/traffic.json profiles/${p%%_*}_pmc_traffic_bench_${p#*_}.json
cp gpurun_out/sqb/sq.json profiles/${p%%_*}_pmc_sq_bench_${p#*_}.json
[ -f gpurun_out/pmcc/ks/run_kernel_stats.csv ] && cp gpurun_out/pmcc/ks/run_kernel_stats.csv profiles/${p}_concat_kernel_stats.csv
ls -la profiles/${p}* profiles/${p%%_*}_pmc_*_${p#*_}.json
