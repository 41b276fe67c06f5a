"""Mean per-dispatch rocprofv3 counter values by kernel, from one or more
run_counter_collection.csv files (tools/gpu_run.sh pmc passes), with the
kernel-trace duration.  Prints one JSON object per kernel.  Analysis helper."""
import collections
import csv
import json
import sys


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if name.startswith("__amd"):
                continue
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[name]["_us"].append(dur)
            agg[name]["_vgpr"] = [float(r["VGPR_Count"])]
            agg[name]["_lds"] = [float(r["LDS_Block_Size"])]
    for name, d in agg.items():
        out = {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())}
        print(json.dumps({"kernel": name[:80], **out}))


if __name__ == "__main__":
    main(sys.argv[1:])
