"""Diagnostic: static instruction-category count of k_render_tile's phases from the ISA.

Compiles sdhip_tile.hip with -DST_MARK=1 (asm comments ";@T n" at the phase-timer points
and ";@M n" at the item-loop boundaries, no code of their own) to gfx950 assembly, takes
one kernel instance and counts, per marked region in program order, MFMA / VALU / SALU /
LDS / VMEM / wait instructions.  Static counts: a region inside the item loop runs once per
item, the rest once per step.  The scheduler may move arithmetic across the markers, so the
split is approximate.  usage: tile_isa_count.py [P=2] [ZIN=0] [RPW=1] (C2: RPW 1, C1: 2)"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from scenedino_amd import build as b  # noqa: E402

# ST_T(i) closes phase i (sdhip_tile.hip); ST_M(i) opens an item-loop phase
T_PHASE = {0: "ray_pass (next ray)", 1: "head", 2: "itemA(0)", 3: "ray_col", 4: "barrier X",
           5: "stage + tap_addrs", 6: "item loop", 7: "epilogue", 8: "vmcnt", 9: "barrier Y",
           10: "ray pass: z", 11: "ray pass: geo + colour", 12: "ray pass: box"}
M_PHASE = {20: "item A: records + tap bases", 21: "item A: taps (tr reads + MFMA)",
           22: "item A: positional code (frags + MFMA)", 23: "item A: relu / pack X",
           24: "item A: sigma MFMA, softplus, alpha, scan", 25: "(after item A)",
           26: "item B: weight, depth / colour sums", 27: "item B: hidden-space compositing",
           28: "(after item B)"}


def region_name(start, end):
    """A region between two markers: an M marker names what follows it, a T marker what
    precedes it."""
    if start and start[0] == "M":
        return f"{start}: {M_PHASE.get(int(start[1:]), '')}"
    if end and end[0] == "T":
        return f"{end}: {T_PHASE.get(int(end[1:]), '')}"
    return f"{start or 'entry'}..{end or 'end'}"


def cat(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    return "other"


def main():
    kv = dict(a.split("=") for a in sys.argv[1:])
    P, ZIN, RPW = kv.get("P", "2"), kv.get("ZIN", "0"), kv.get("RPW", "1")
    zb = "Lb1E" if ZIN == "1" else "Lb0E"
    sym = f"_Z13k_render_tileILi{P}E{zb}Li8ELi{RPW}EEv7st_args:"
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "t.s")
        flags = [f for f in b.FLAGS if not f.startswith("--offload-arch")]
        subprocess.run([b.hipcc(), "--offload-arch=gfx950", "--cuda-device-only", "-S"] + flags +
                       ["-DST_MARK=1", "-o", out, os.path.join(b.HERE, "csrc", "sdhip_tile.hip")],
                       check=True, cwd=td)
        lines = open(out).read().split("\n")
    i0 = next(i for i, l in enumerate(lines) if l.startswith(sym))
    i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
    regs, cur = [], [None, None, {}]
    regs.append(cur)
    for l in lines[i0:i1 + 1]:
        m = re.search(r";@([TM]) (\d+)", l)
        if m:
            cur[1] = m.group(1) + m.group(2)
            cur = [cur[1], None, {}]
            regs.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "_")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = cat(op)
        cur[2][c] = cur[2].get(c, 0) + 1
    cols = ["mfma", "valu", "salu", "lds", "vmem", "wait", "other"]
    print(f"k_render_tile<P={P}, ZIN={ZIN}, NW=8, RPW={RPW}>: static instructions per region "
          "(program order)")
    print(f"{'region':48s}" + "".join(f"{c:>7s}" for c in cols))
    tot = {}
    for start, end, d in regs:
        if not d:
            continue
        label = region_name(start, end)
        print(f"{label[:48]:48s}" + "".join(f"{d.get(c, 0):7d}" for c in cols))
        for c in cols:
            tot[c] = tot.get(c, 0) + d.get(c, 0)
    print(f"{'total':48s}" + "".join(f"{tot.get(c, 0):7d}" for c in cols))


if __name__ == "__main__":
    main()
