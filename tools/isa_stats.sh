#!/usr/bin/env bash
# Static ISA statistics of the sweep kernels (cross-compiled for gfx950, no GPU).
# usage: tools/isa_stats.sh [extra hipcc -D flags ...]
# Prints per-kernel VGPR/SGPR/scratch/LDS/occupancy and an opcode histogram
# of the ECS exact kernel (top 30 opcodes).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/pht_isa
mkdir -p "$OUT"
cd "$OUT"
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -ffp-contract=off -Wno-pass-failed \
  -DPHT_DETMATH_LDS "$@" -I"$ROOT/include" -I"$ROOT/phasetype_amd/csrc" \
  --cuda-device-only -S -o k.s -DPHT_NT=${PHT_NT:-10} "$ROOT/phasetype_amd/csrc/pht_kernels_nt.hip"
python3 - k.s <<'EOF'
import re, sys, collections
s = open(sys.argv[1]).read()
# resource usage comments emitted per function
for blk in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S | re.M):
    name, body = blk.group(1), blk.group(2)
    if "ecs_exact" not in name and "sweep_kernel" not in name:
        continue
    ops = collections.Counter()
    for line in body.splitlines():
        t = line.strip()
        if not t or t.startswith((";", ".", "_", "s_nop")) or t.endswith(":"):
            continue
        ops[t.split()[0]] += 1
    tot = sum(ops.values())
    print(f"{name}: {tot} static insts")
    if "ecs_exact" in name and "Lb0" in name:
        for op, c in ops.most_common(30):
            print(f"   {op:28s} {c}")
# per-kernel resources (the comment block after each function body)
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)\.Lfunc_end.*?; NumVgprs: (\d+).*?; ScratchSize: (\d+).*?; Occupancy: (\d+)",
                     s, re.S | re.M):
    print(f"  {m.group(1)[:60]:60s} vgpr {m.group(3):>4s} scratch {m.group(4):>5s} occ {m.group(5)}")
EOF
