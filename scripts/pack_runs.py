#!/usr/bin/env python3
"""Pack a profile folder's per-run bench.py JSON lines (one file per run) into one runs.jsonl:
each line {"file": the run's file name, "line": its JSON}; the single files are removed.  Tables
(table.txt), logs and diffs stay as they are.  Keeps the evidence one file per A/B.
Usage: python3 scripts/pack_runs.py DIR..."""
import glob
import json
import os
import sys


def pack(d):
    files = sorted(f for f in glob.glob(os.path.join(d, "*.json")))
    if not files:
        return 0
    out = os.path.join(d, "runs.jsonl")
    with open(out, "a") as o:
        for f in files:
            try:
                line = json.load(open(f))
            except ValueError:
                continue
            o.write(json.dumps({"file": os.path.basename(f), "line": line}) + "\n")
            os.remove(f)
    return len(files)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(d, pack(d))
