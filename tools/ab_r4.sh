#!/bin/bash
# Same-box A/B of the working build against ldpc_sparc_amd/_lib_alt
# (tools/build_alt.sh) -- or, with OLD_ENV="VAR=value", against the working
# build under that environment setting -- interleaved twice, on the bench
# lines named by $1:
#   c2     C2 + the R=1.3 companion (no CPU legs)
#   concat C5 only
#   bp     C3 only
#   sc     C4 + notebook
# with the parity tests of $2 (pytest paths, optional) first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_$1; rm -rf $O; mkdir -p $O
case $1 in
  c2) ARGS="--no-bp --no-sc --no-sc-notebook --no-concat --no-f64";;
  concat) ARGS="--no-bp --no-sc --no-sc-notebook --no-r13 --no-f64 --steps 1 --warmup 1";;
  bp) ARGS="--no-sc --no-sc-notebook --no-concat --no-r13 --no-f64 --bp-ebn0-extra --steps 1 --warmup 1";;
  sc) ARGS="--no-bp --no-concat --no-r13 --no-f64 --steps 1 --warmup 1";;
esac
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
fi
for i in 1 2; do
  if [ -n "$OLD_ENV" ]; then
    env $OLD_ENV timeout -k 10 300 python bench.py $ARGS --cpu-seconds 0 > $O/old$i.json 2>$O/old$i.err
  else
    LDPC_SPARC_AMD_LIB=$PWD/ldpc_sparc_amd/_lib_alt/libldpc_sparc_amd.so timeout -k 10 300 python bench.py $ARGS --cpu-seconds 0 > $O/old$i.json 2>$O/old$i.err
  fi
  timeout -k 10 300 python bench.py $ARGS --cpu-seconds 0 > $O/new$i.json 2>$O/new$i.err
done
python3 tools/ab_summary.py $O > $O/summary.txt
cat $O/summary.txt
