"""Tile anonymiser restatement (oracle/tiles_oracle.py) against the reference's own
report() outputs (tests/golden/tiles_golden.json, make_tiles_golden.py)."""
import json
import os
import random

import tiles_oracle as to

GOLD = os.path.join(os.path.dirname(__file__), "golden", "tiles_golden.json")


def _golden():
    with open(GOLD) as f:
        return json.load(f)["cases"]


def test_cull_matches_reference_report():
    cases = _golden()
    assert len(cases) > 1000
    for c in cases:
        assert to.tile_body(c["lines"], c["privacy"]) == c["body"]


def test_group_rule_equals_cull_loop():
    """cull_by_groups (the form the GPU evaluates) == the reference loop."""
    for c in _golden():
        srt = sorted(c["lines"])
        keys = [tuple(l.split(",")[:2]) for l in srt]
        sizes, order = [], []
        for k in keys:
            if order and order[-1] == k:
                sizes[-1] += 1
            else:
                order.append(k)
                sizes.append(1)
        keep = to.cull_by_groups(sizes, c["privacy"])
        want = [l for l, k in zip(srt, keys) if keep[order.index(k)]]
        assert want == to.privacy_cull(c["lines"], c["privacy"])
    rng = random.Random(5)
    for _ in range(3000):
        sizes = [rng.choice([1, 1, 2, 3, 5]) for _ in range(rng.randrange(1, 7))]
        lines = ["%d,0,x%d\n" % (g, k) for g, n in enumerate(sizes) for k in range(n)]
        p = rng.randrange(1, 6)
        keep = to.cull_by_groups(sizes, p)
        assert [l for l in lines if keep[int(l.split(",")[0])]] == to.privacy_cull(lines, p)


def test_windows_and_buckets():
    # inactivity windows (simple_reporter.py:151-160): gaps > 120 split, < 2 points skipped
    t = [0, 10, 20, 200, 500, 510, 1000]
    assert to.windows(t, 120) == [(0, 3), (4, 6)]
    assert to.windows([5], 120) == []
    assert to.windows([0, 120, 240], 120) == [(0, 3)]        # a gap of exactly 120 does not split
    u = ["b", "a", "b", "a", "a"]
    tm = [30, 5, 10, 400, 7]
    assert to.split_windows(u, tm, 120) == [("a", [1, 4]), ("b", [2, 0])]
    # hour buckets and rows (simple_reporter.py:176-196)
    rep = [{"id": 1 | (5 << 3), "next_id": 2, "t0": 3590.4, "t1": 3650.5, "length": 500, "queue_length": 0},
           {"id": 2, "t0": 100.0, "t1": 100.4, "length": 5, "queue_length": 0},            # dt <= 0.5: dropped
           {"id": 2 | (7 << 3), "t0": 7300.0, "t1": 7330.5, "length": 300, "queue_length": 4}]
    tiles = to.tile_lines(rep, 3500, 7400, 3600, "src", "auto")
    assert sorted(tiles) == ["0_3599/1/5", "3600_7199/1/5", "7200_10799/2/7"]
    assert tiles["0_3599/1/5"] == ["%d,2,60,1,500,0,3590,3651,src,AUTO\n" % (1 | (5 << 3))]
    assert tiles["7200_10799/2/7"] == ["%d,%d,31,1,300,4,7300,7331,src,AUTO\n" % (2 | (7 << 3), to.INVALID_SEGMENT_ID)]
    assert to.py2_round(30.5) == 31 and to.py2_round(2.5) == 3
