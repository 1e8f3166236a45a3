#!/bin/bash
# Register spills of every kernel in the library: each .hip compiled to
# assembly with the Makefile's flags; prints kernels with VGPR or SGPR spills.
cd "$(dirname "$0")/.." || exit 1
O=${TMPDIR:-/tmp}/spill_check; mkdir -p $O
for f in ldpc_sparc_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  extra=""
  case $b in bp) extra="-ffp-contract=off";; bp_grouped) extra="-ffp-contract=off -fno-honor-nans";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude --cuda-device-only -S -x hip $extra $f -o $O/$b.s 2>/dev/null &
done
wait
python3 - $O <<'PY'
import glob, re, sys
bad = 0
for f in sorted(glob.glob(sys.argv[1] + "/*.s")):
    s = open(f).read()
    if "amdhsa.kernels" not in s:
        continue
    for blk in s[s.index("amdhsa.kernels"):].split("  - .")[1:]:
        nm = re.search(r"\.name:\s+(\S+)", blk)
        vs = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
        ss = re.search(r"\.sgpr_spill_count:\s+(\d+)", blk)
        if nm and vs and ss and (int(vs.group(1)) or int(ss.group(1))):
            bad += 1
            print(f"{f.split('/')[-1][:-2]:12s} {nm.group(1)[:90]:90s} vgpr_spill {vs.group(1):>3s} sgpr_spill {ss.group(1):>3s}")
print(f"{bad} kernels with spills")
PY
