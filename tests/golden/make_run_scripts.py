"""Fixture generator (run in the build container, where /root/reference exists):
the Photogrammetrie command line of every run-scripts/run-*.sh of the reference,
tokenised as bash would (the scripts hold only plain words and $1/$2), written to
tests/golden/run_scripts.json.  The fixture is data (argument lists); the replay
test (tests/test_cli.py) substitutes $1/$2 and runs them through sfmx's CLI."""
import glob
import json
import os
import shlex

REF = "/root/reference/run-scripts"
out = {}
for path in sorted(glob.glob(os.path.join(REF, "run-*.sh"))):
    for line in open(path):
        line = line.strip()
        if not line.startswith("Photogrammetrie "):
            continue
        words = shlex.split(line.split("|")[0])
        out[os.path.basename(path)] = words
json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "run_scripts.json"), "w"), indent=1)
print(len(out), "scripts")
