"""Extract the one Match input the reference holds: the 14-point Manila trace of
/root/reference/README.md:269 (the /report example link), as a JSON fixture (data only).

    python tests/golden/make_manila_fixture.py      # run in the build container

The README gives no expected output, only the reply schema (README.md:270-301); the GPU test
(tests/test_gpu_manila.py) checks the engine's reply against the oracle and that schema."""
import json
import os
import re
import urllib.parse

HERE = os.path.dirname(os.path.abspath(__file__))
README = "/root/reference/README.md"

text = open(README, encoding="utf-8").read().splitlines()
line = text[268]   # README.md:269 (1-based)
m = re.search(r"report\?json=(\{.*\})\]\(", line) or re.search(r"report\?json=(\{.*\})\)", line)
req = json.loads(urllib.parse.unquote(m.group(1)))
assert req["uuid"] == "100609" and len(req["trace"]) == 14
out = {"source": "reference README.md:269 (/report example link)", "request": req}
with open(os.path.join(HERE, "manila_readme_trace.json"), "w") as f:
    json.dump(out, f, indent=1)
print("wrote", len(req["trace"]), "points")
