#!/usr/bin/env python3
"""Static ISA attribution of the ECS exact kernel to its stamped phases
(VERDICT r05 item 1).  Diagnostic, CPU only, never run on a GPU.

A -D PHT_ISA_MARKS compile turns every PHT_STAMP(ln, k) into the assembly
comment "; @phase k" (pht_device.h).  This script compiles one kernel unit
(pht_kernels_nt.hip at compile-time n) to gfx950 assembly with the product
flags, splits the chosen kernel into basic blocks, and gives every
instruction the phase(s) whose marker reaches it through the control-flow
graph without crossing another marker (a block reached from two markers is
split between them).  The code after marker k runs until the next stamp,
which adds its time to that stamp's slot (tools/stamps.py names): the round
order is 12, 1, 2, ..., 11 inside ecs_round, then 0 at the loop's top, so
the code after marker k is named after CLOSES[k].  Instructions are classed VALU-FP64 (every v_*_f64
opcode, incl. compares and conversions), VALU-other, SALU, LDS, VMEM
(global/buffer/scratch/flat), SMEM, branch/wait (s_cbranch, s_branch,
s_waitcnt, s_nop, ...).

usage: python3 tools/isa_phases.py [--nt 10] [--kernel ecs_exact_kernelILi10ELb0ELb0EE] [--json out.json]
       [--s existing.s]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

NAMES = {0: "phaseA_absorb_newobs", 12: "topup", 1: "dens_load_E0", 2: "start_init4", 3: "pend_insert",
         4: "meets", 5: "cumulate", 6: "f0_cap", 7: "invert_u", 8: "proposal_eval", 9: "test_metropolis",
         10: "big_general", 11: "finish_movemass"}
# the stamp that closes the code after each marker (pht_kernels_impl.h /
# pht_ecs_round.h stamp order: ... 11 -> (loop) 0 -> 12 -> 1 -> ... -> 11)
CLOSES = {12: 1, 1: 2, 2: 3, 3: 4, 4: 5, 5: 6, 6: 7, 7: 8, 8: 9, 9: 10, 10: 11, 11: 0, 0: 12}
CATS = ["valu_f64", "valu_other", "salu", "lds", "vmem", "smem", "branch_wait"]


def category(op):
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache", "s_memtime", "s_memrealtime")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_endpgm", "s_barrier", "s_setprio",
                      "s_sleep", "s_setpc", "s_swappc", "s_getpc", "s_trap", "s_sethalt", "s_delay")):
        return "branch_wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu_f64" if "f64" in op else "valu_other"
    return "other"


def compile_s(nt, out):
    import phasetype_amd.build as B

    flags = list(B.UNIT_FLAGS.get(nt, ()))
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
           "-Wno-pass-failed", "-DPHT_DETMATH_LDS", "-DPHT_ISA_MARKS", f"-DPHT_NT={nt}",
           f"-I{os.path.join(REPO, 'include')}", f"-I{os.path.join(REPO, 'phasetype_amd', 'csrc')}",
           "--cuda-device-only", "-S", "-o", out] + flags + [os.path.join(REPO, "phasetype_amd", "csrc",
                                                                        "pht_kernels_nt.hip")]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def function_lines(s, kernel):
    lines = s.splitlines()
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^_Z\S*" + re.escape(kernel) + r"\S*:", ln):
            start = i
        elif start is not None and ln.startswith(".Lfunc_end"):
            return lines[start + 1:i]
    raise SystemExit(f"kernel {kernel} not found")


def parse(lines):
    """basic blocks: list of dicts {label, items: [("m", k) | ("i", op, text)], succ: [labels], fall}"""
    blocks = []
    cur = {"label": None, "items": [], "succ": [], "fall": True}
    blocks.append(cur)

    def new(label):
        nonlocal cur
        cur = {"label": label, "items": [], "succ": [], "fall": True}
        blocks.append(cur)

    for raw in lines:
        t = raw.strip()
        if not t:
            continue
        m = re.match(r"^(\.LBB\S+):", t)
        if m:
            new(m.group(1))
            continue
        m = re.match(r"^; @phase (\d+)", t)
        if m:
            cur["items"].append(("m", int(m.group(1))))
            continue
        m = re.match(r"^; @sub (\S+)", t)
        if m:
            cur["items"].append(("s", m.group(1)))
            continue
        if t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cur["items"].append(("i", op, t))
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = t.split()[-1]
            cur["succ"].append(tgt)
            if op == "s_branch":
                cur["fall"] = False
            new(None)
        elif op == "s_endpgm":
            cur["fall"] = False
            new(None)
    return [b for b in blocks if b["items"] or b["label"]]


def attribute(blocks):
    idx = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
    succs = []
    for i, b in enumerate(blocks):
        s = [idx[t] for t in b["succ"] if t in idx]
        if b["fall"] and i + 1 < len(blocks):
            s.append(i + 1)
        succs.append(s)
    owners = collections.defaultdict(set)  # (block, item) -> phases
    variant = collections.defaultdict(set)  # (block, item) -> sub-variant tags

    def walk(tag, bi, start, dest, stop_at_sub):
        """mark the instructions reachable from (bi, start) up to the next phase
        marker; a sub-variant walk (stop_at_sub) also ends at its own "end",
        passing through nested sub-regions (their depth is tracked)"""
        stack = [(bi, start, 0)]
        seen = set()
        while stack:
            b, st, depth = stack.pop()
            if (b, st, depth) in seen:
                continue
            seen.add((b, st, depth))
            stopped = False
            for k in range(st, len(blocks[b]["items"])):
                it = blocks[b]["items"][k]
                if it[0] == "m":
                    stopped = True
                    break
                if it[0] == "s" and stop_at_sub:
                    if it[1] == "end":
                        if depth == 0:
                            stopped = True
                            break
                        depth -= 1
                    else:
                        depth += 1
                    continue
                if it[0] == "i":
                    dest[(b, k)].add(tag)
            if not stopped:
                for nb in succs[b]:
                    stack.append((nb, 0, depth))

    walk("setup", 0, 0, owners, False)
    for bi, b in enumerate(blocks):
        for k, it in enumerate(b["items"]):
            if it[0] == "m":
                walk(CLOSES.get(it[1], it[1]), bi, k + 1, owners, False)
            elif it[0] == "s" and it[1] != "end":
                walk(it[1], bi, k + 1, variant, True)
    table = collections.defaultdict(lambda: collections.Counter())
    ops = collections.defaultdict(collections.Counter)
    for bi, b in enumerate(blocks):
        for k, it in enumerate(b["items"]):
            if it[0] != "i":
                continue
            ph = owners.get((bi, k)) or {"unreached"}
            vs = variant.get((bi, k)) or set()
            v = "+".join(sorted(vs)) if vs else "common"
            w = 1.0 / len(ph)
            for p in ph:
                if True:
                    key = p if v == "common" else (p, v)
                    table[key][category(it[1])] += w
                    table[key]["total"] += w
                    ops[key][it[1]] += w
    OWN.update(owners)
    VAR.update(variant)
    return table, ops


OWN, VAR = {}, {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nt", type=int, default=10)
    ap.add_argument("--kernel")
    ap.add_argument("--s", help="an existing PHT_ISA_MARKS assembly file")
    ap.add_argument("--json")
    ap.add_argument("--weights", help="variant frequencies per wave-round, e.g. c9=0.05,c11=0.77,c13=0.18")
    ap.add_argument("--dump", help="print the instructions of this phase (its name)")
    ap.add_argument("--variant", help="with --dump: only this sub-variant (or 'common')")
    ap.add_argument("--top", type=int, default=0, help="top opcodes per phase")
    a = ap.parse_args()
    kernel = a.kernel or f"ecs_exact_kernelILi{a.nt}ELb0ELb0EE"
    path = a.s
    if not path:
        path = os.path.join(tempfile.mkdtemp(prefix="pht_isa_"), f"k{a.nt}.s")
        compile_s(a.nt, path)
    blocks = parse(function_lines(open(path).read(), kernel))
    table, ops = attribute(blocks)
    order = ["setup", 0, 12, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, "unreached"]
    weights = {}
    for kv in (a.weights or "").split(","):
        if "=" in kv:
            k, v = kv.split("=")
            weights[k] = float(v)
    rows = []
    print(f"{'phase':30s} " + " ".join(f"{c:>11s}" for c in CATS + ["total"]))
    for p in order:
        keys = [k for k in table if k == p or (isinstance(k, tuple) and k[0] == p)]
        if not keys:
            continue
        name = NAMES.get(p, str(p)) if p != "setup" else "setup"
        dyn = collections.Counter()
        for key in sorted(keys, key=str):
            label = name if key == p else f"  {name}[{key[1]}]"
            r = {"phase": name, "variant": None if key == p else key[1],
                 **{c: round(table[key][c], 1) for c in CATS + ["total"]}}
            if a.top:
                r["top"] = [(o, round(c, 1)) for o, c in ops[key].most_common(a.top)]
            rows.append(r)
            print(f"{label:30s} " + " ".join(f"{table[key][c]:11.1f}" for c in CATS + ["total"]))
            if a.top:
                print("    " + ", ".join(f"{o} {c:.0f}" for o, c in ops[key].most_common(a.top)))
            wv = 1.0
            if key != p:
                for t in key[1].split("+"):
                    wv *= weights.get(t, 0.0)
            for c in CATS + ["total"]:
                dyn[c] += wv * table[key][c]
        if len(keys) > 1 and weights:
            rows.append({"phase": name, "variant": "weighted", **{c: round(dyn[c], 1) for c in CATS + ["total"]}})
            print(f"{'  ' + name + '[weighted]':30s} " + " ".join(f"{dyn[c]:11.1f}" for c in CATS + ["total"]))
    if a.dump is not None:
        for bi, b in enumerate(blocks):
            for k, it in enumerate(b["items"]):
                if it[0] == "i" and a.dump in {str(NAMES.get(p, p)) for p in (OWN.get((bi, k)) or ())} and \
                        (a.variant is None or a.variant in (VAR.get((bi, k)) or {"common"})):
                    print(it[2])
    if a.json:
        json.dump({"kernel": kernel, "nt": a.nt, "rows": rows}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
