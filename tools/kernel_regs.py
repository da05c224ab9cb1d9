#!/usr/bin/env python3
"""Register / spill / scratch metadata of every gfx950 kernel in a built
libPhaseType.so (no GPU): the .hip_fatbin offload bundles are split into
their code objects and each object's AMDGPU metadata note is read with
llvm-readelf.  vgpr = arch + acc VGPRs per lane (512 per SIMD lane on gfx950:
occupancy = 512 // vgpr waves per SIMD, at most 8).

usage: python3 tools/kernel_regs.py [lib.so] [--filter SUBSTR ...]
"""
import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(so):
    ro = subprocess.run([f"{LLVM}/llvm-readelf", "-S", "-W", so], capture_output=True, text=True, check=True).stdout
    off = size = None
    for line in ro.splitlines():
        if ".hip_fatbin" in line:
            f = line.split("]")[1].split()
            off, size = int(f[3], 16), int(f[4], 16)
    if off is None:
        raise SystemExit(f"{so}: no .hip_fatbin section")
    with open(so, "rb") as fh:
        fh.seek(off)
        data = fh.read(size)
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = 0
    while True:
        i = data.find(magic, pos)
        if i < 0:
            break
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                yield data[i + o:i + o + sz]
        pos = i + len(magic)


def kernels(so):
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(so)):
            path = os.path.join(td, f"co{k}.elf")
            with open(path, "wb") as fh:
                fh.write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", path], capture_output=True, text=True,
                                   check=True).stdout
            for blk in re.split(r"\n  - \.agpr_count:", notes)[1:]:
                def g(key):
                    m = re.search(r"\." + key + r":\s+(\S+)", blk)
                    return int(m.group(1)) if m and m.group(1).isdigit() else (m.group(1) if m else None)
                name = g("name")
                out[name] = {"vgpr": g("vgpr_count"), "agpr": int(blk.split()[0]), "vgpr_spill": g("vgpr_spill_count"),
                             "sgpr_spill": g("sgpr_spill_count"), "scratch": g("private_segment_fixed_size"),
                             "lds_static": g("group_segment_fixed_size")}
                v = out[name]["vgpr"] or 1
                out[name]["waves_per_simd"] = min(8, 512 // max(v, 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(REPO, "phasetype_amd", "_lib", "libPhaseType.so"))
    ap.add_argument("--filter", nargs="*", default=[])
    a = ap.parse_args()
    ks = kernels(a.lib)
    for name in sorted(ks):
        if a.filter and not any(f in name for f in a.filter):
            continue
        d = ks[name]
        print(f"{name[:70]:70s} vgpr {d['vgpr']:>3} (acc {d['agpr']:>3}) waves {d['waves_per_simd']} "
              f"vspill {d['vgpr_spill']:>4} scratch {d['scratch']:>5}")


if __name__ == "__main__":
    sys.exit(main())
