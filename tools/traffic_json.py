#!/usr/bin/env python3
"""Per-dispatch HBM traffic of the render-path kernels from rocprofv3 PMC passes
(tools/profile.sh: FETCH_SIZE and WRITE_SIZE in separate passes), corrected as
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes: FETCH_SIZE / WRITE_SIZE
are KB; on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane reads, so it is
doubled; WRITE_SIZE is taken as is.  usage: traffic_json.py gpurun_out/prof_TAG out.json"""
import collections
import csv
import glob
import json
import os
import sys

d, out = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        for k in ("k_render_tile", "k_render_proj", "k_project", "k_head_hc", "k_render<", "k_field_gather_bwd",
                  "k_field_gather", "k_composite_bwd", "k_unpack_grid", "k_pack_grid",
                  "k_mlp_fwd", "k_mlp_bwd", "k_mlp_wgrad", "k_mw_split", "k_mw_final", "k_wgrad",
                  "k_composite", "k_seg_head", "k_ssc_confusion",
                  "k_attn_lds", "k_attn_dir", "k_grow3", "k_field"):
            if k in name:
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                break
res = {"source": d, "note": "per-dispatch means; bytes = 2 x FETCH_SIZE(KB) x 1024 + "
       "WRITE_SIZE(KB) x 1024 (MI355X_MICROARCH.md HBM/rocprofv3 corrections)", "kernels": {}}
for k, c in vals.items():
    fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) * 1024 if c.get("FETCH_SIZE") else None
    write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) * 1024 if c.get("WRITE_SIZE") else None
    res["kernels"][k] = {"fetch_size_bytes_raw": fetch, "write_size_bytes": write,
                         "hbm_bytes": (2 * fetch + write) if fetch is not None and write is not None
                         else None}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
