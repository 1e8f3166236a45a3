#!/bin/bash
# tools/amp_probe.py at precision $1 under each environment setting of the
# remaining arguments ("-" = none), interleaved twice:
#   bash tools/amp_env_sweep.sh f64 - SG_AMP_STAGGER=20000 SG_AMP_PMAX=4096
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=$1; shift
for rep in 1 2; do
  for e in "$@"; do
    if [ "$e" = "-" ]; then E=""; else E="$e"; fi
    echo "$e: $(env $E timeout -k 10 300 python tools/amp_probe.py 256 $P)"
  done
done
