#!/bin/bash
# Per-kernel resources of the gfx950 device build (VGPRs, scratch bytes/lane, LDS, occupancy), one line each.
# usage: tools/res_usage.sh [source dir (default: this tree's csrc)] [extra hipcc flags...]
SRC=${1:-$(dirname "$0")/../isaacgym-hand-arm_amd/csrc}
shift
INC=$(cd "$SRC/../../include" && pwd)
out=$(mktemp)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC --cuda-device-only -c \
    -Rpass-analysis=kernel-resource-usage -I "$INC" "$@" "$SRC/handarm_hip.hip" -o /dev/null 2> "$out"
python3 - "$out" <<'PY'
import re, sys
cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}; rows.append(cur); continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    if r.get("vgpr", 0) >= 60:
        print(f"{r['name']:28s} vgpr {r.get('vgpr')} scratch {r.get('scratch')} lds {r.get('lds')} occ {r.get('occ')}")
PY
rm -f "$out"
