"""The coalescer's failure policy (reporter_amd/csrc/serve_policy.hpp), on the host.

ADVICE r02: a whole-batch failure that repeats (a device error, a route-table build that
cannot fit) must be attempted once, not re-run by bisection 2n-1 times; only a batch too large
for the device is split, within a fixed retry budget.  The policy is header-only and is driven
here by a fake runner compiled with g++ (no GPU)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_serve_policy(tmp_path):
    exe = str(tmp_path / "serve_policy_test")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "reporter_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "serve_policy_test.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "serve policy ok" in r.stdout
