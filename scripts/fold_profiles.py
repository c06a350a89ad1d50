"""Fold one round's per-run profile files into one archive per experiment (VERDICT r4
item 7): profiles/rNN_vMM_<name>.<ext> -> profiles/rNN_vMM.json, {"experiment", "files":
{<original file name>: parsed JSON | text}}.  rocprofv3 kernel-trace summaries
(*kernel_stats.csv) and PMC summaries (*pmc_<config>.json, read by bench.py) stay as
files.  A citation `rNN_vMM_<name>` in DESIGN.md is the entry of that name in the archive.
Usage: python3 scripts/fold_profiles.py r04"""
import collections
import json
import re
import sys
from pathlib import Path

root = Path(__file__).resolve().parent.parent / "profiles"
rnd = sys.argv[1]
keep = re.compile(r"(kernel_stats\.csv|pmc_c\d\.json)$")
groups = collections.defaultdict(list)
for f in sorted(root.iterdir()):
    m = re.match(rf"({rnd}_v\d+)_", f.name)
    if m and not keep.search(f.name):
        groups[m.group(1)].append(f)
for exp, files in sorted(groups.items()):
    out = root / f"{exp}.json"
    arch = json.loads(out.read_text()) if out.exists() else {"experiment": exp, "files": {}}
    for f in files:
        text = f.read_text(errors="replace")
        try:
            val = json.loads(text)
        except ValueError:
            lines = [ln for ln in text.splitlines() if ln.strip()]
            try:  # JSON lines
                val = [json.loads(ln) for ln in lines]
            except ValueError:
                val = text
        arch["files"][f.name] = val
    out.write_text(json.dumps(arch, indent=1) + "\n")
    for f in files:
        f.unlink()
    print(exp, len(files), "->", out.name)
