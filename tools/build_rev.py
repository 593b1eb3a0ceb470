"""Diagnostic: build libsdhip.so from the HIP sources of another git revision into
scenedino_amd/variants/<name>.so (same flags as scenedino_amd/build.py) -- the A side of an
interleaved A/B against the working tree (tools/gpu_session.sh ab:CFG:<name>:REPS).
usage: build_rev.py <rev> <name> [-DX=1 ...]"""
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from scenedino_amd import build as b  # noqa: E402

rev, name, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
tmp = tempfile.mkdtemp(prefix="sdrev_")
files = subprocess.run(["git", "ls-tree", "-r", "--name-only", rev, "scenedino_amd/csrc", "include"],
                       cwd=ROOT, check=True, capture_output=True, text=True).stdout.split()
for f in files:
    dst = os.path.join(tmp, f)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "wb") as fh:
        fh.write(subprocess.run(["git", "show", f"{rev}:{f}"], cwd=ROOT, check=True,
                                capture_output=True).stdout)
od = os.path.join(b.HERE, "variants", "_obj_" + name)
os.makedirs(od, exist_ok=True)


def one(src):
    o = os.path.join(od, os.path.basename(src) + ".o")
    subprocess.run([b.hipcc()] + b.FLAGS + defs + ["-c", "-o", o, os.path.join(tmp, "scenedino_amd", src)],
                   check=True)
    return o


srcs = [s for s in b.SOURCES if os.path.exists(os.path.join(tmp, "scenedino_amd", s))]
with ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(one, srcs))
out = os.path.join(b.HERE, "variants", name + ".so")
subprocess.run([b.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
print(out)
