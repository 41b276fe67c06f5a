"""Mean per-dispatch rocprofv3 counter values by kernel, from one or more
run_counter_collection.csv files (tools/gpu_run.sh pmc passes), with the
kernel-trace duration.  Prints one JSON object per kernel.  `--skip N` drops
each kernel's first N dispatches (warm-up / clock transient).  Analysis helper."""
import collections
import csv
import json
import sys


def main(paths, skip=0):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        order = collections.defaultdict(list)       # kernel -> its dispatch ids in order
        for r in rows:
            if r["Dispatch_Id"] not in order[r["Kernel_Name"]]:
                order[r["Kernel_Name"]].append(r["Dispatch_Id"])
        for r in rows:
            name = r["Kernel_Name"]
            if name.startswith("__amd") or order[name].index(r["Dispatch_Id"]) < skip:
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
    args = sys.argv[1:]
    nskip = 0
    if args and args[0] == "--skip":
        nskip, args = int(args[1]), args[2:]
    main(args, nskip)
