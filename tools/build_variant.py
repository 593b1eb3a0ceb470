"""Diagnostic: build libsdhip.so with extra -D switches into scenedino_amd/variants/<name>.so
(same sources and flags as scenedino_amd/build.py).  usage: build_variant.py name -DA=1 ..."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from scenedino_amd import build as b  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
od = os.path.join(b.HERE, "variants", "_obj_" + name)
os.makedirs(od, exist_ok=True)
objs = []


def one(src):
    o = os.path.join(od, os.path.basename(src) + ".o")
    subprocess.run([b.hipcc()] + b.FLAGS + defs + ["-c", "-o", o, os.path.join(b.HERE, src)], check=True)
    return o


with ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(one, b.SOURCES))
out = os.path.join(b.HERE, "variants", name + ".so")
subprocess.run([b.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
print(out)
