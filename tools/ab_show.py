import glob, json, sys
for tag in ("base", "new"):
    v = [json.load(open(f))["value"] for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.json"))]
    print(tag, v, "mean %.1f" % (sum(v) / max(1, len(v))))
