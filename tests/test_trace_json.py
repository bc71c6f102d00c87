"""The /report boundary's single-pass request reader and reply formatter (trace_json.hpp), on
the host: over ~27k generated requests, mutations and every prefix of small documents it returns
exactly what the DOM reader path returned (points bit for bit, options, or the same error
message), and to_chars replies parse back to the doubles "%.17g" gives (tests/cpp/trace_json_test.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trace_json_reader_matches_dom_reader(tmp_path):
    exe = str(tmp_path / "trace_json_test")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-ffp-contract=off",
                    "-I" + os.path.join(ROOT, "reporter_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "trace_json_test.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "trace json ok" in r.stdout
