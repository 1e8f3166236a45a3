#!/bin/bash
# Builds the library of git revision $1 (default HEAD) in a scratch worktree
# and copies it to ldpc_sparc_amd/_lib_alt/ for same-box A/B runs
# (tools/ab_r4.sh loads it through LDPC_SPARC_AMD_LIB).
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
W=${TMPDIR:-/tmp}/sg_alt_$(git rev-parse --short $rev)
[ -d $W ] || git worktree add --detach $W $rev >/dev/null
make -s -j8 -C $W/ldpc_sparc_amd/csrc >/dev/null
mkdir -p ldpc_sparc_amd/_lib_alt
cp $W/ldpc_sparc_amd/_lib/libldpc_sparc_amd.so ldpc_sparc_amd/_lib_alt/
echo "ldpc_sparc_amd/_lib_alt <- $rev ($(git rev-parse --short $rev))"
