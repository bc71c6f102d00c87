"""GPU batch-pipeline stages around the matcher, against the CPU restatements.

  run_points  raw per-vehicle points in arbitrary order -> windows (simple_reporter.py:137-164)
  tiles       valid reports -> hour tiles -> privacy cull -> CSV (simple_reporter.py:176-254)

The oracle side is tiles_oracle.split_windows + the C matcher oracle + report() restatement
+ tiles_oracle.tile_lines / tile_body (the last pinned by the reference's own report()).
Exactness bar: windows and every matcher stage bit-exact; tile files byte-identical.
"""
import json

import numpy as np
import pytest

import meili_oracle as mo
import tiles_oracle as to
from parity_util import compare_all
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu


def _stream(path, n_veh=40, n_pts=240, seed=3):
    """Each vehicle drives two windows separated by a gap > 120 s, plus a lone point after
    another gap (a 1-point window, skipped); all points shuffled."""
    tr = world.generate_traces(path, n_traces=2 * n_veh, n_points=n_pts, rate_s=1.0, noise_m=5.0, seed=seed)
    uu, tm, lo, la, ac = [], [], [], [], []
    for v in range(n_veh):
        t_shift = 0.0
        for part in (2 * v, 2 * v + 1):
            o0, o1 = tr["trace_off"][part], tr["trace_off"][part + 1]
            t = tr["time"][o0:o1] - tr["time"][o0] + 1483300000.0 + 3000.0 * (v % 5) + t_shift
            t_shift = float(t[-1] - 1483300000.0 - 3000.0 * (v % 5)) + 121.0 + (v % 3) * 50
            uu.append(np.full(o1 - o0, v)); tm.append(t); lo.append(tr["lon"][o0:o1]); la.append(tr["lat"][o0:o1])
            ac.append(tr["accuracy"][o0:o1])
        uu.append(np.array([v])); tm.append(np.array([tm[-1][-1] + 500.0]))
        lo.append(np.array([lo[-1][-1]])); la.append(np.array([la[-1][-1]])); ac.append(np.array([ac[-1][-1]]))
    d = dict(uuid=np.concatenate(uu).astype(np.uint32), time=np.concatenate(tm), lon=np.concatenate(lo),
             lat=np.concatenate(la), accuracy=np.concatenate(ac).astype(np.float32))
    perm = np.random.default_rng(seed).permutation(len(d["uuid"]))
    return {k: v[perm] for k, v in d.items()}


def _oracle(g, pts, inactivity=120, opts=None):
    wins = to.split_windows(list(pts["uuid"]), list(pts["time"]), inactivity)
    idx = np.concatenate([np.array(w, np.int64) for _, w in wins])
    off = np.zeros(len(wins) + 1, np.uint32)
    off[1:] = np.cumsum([len(w) for _, w in wins])
    tr = dict(trace_off=off, lon=pts["lon"][idx], lat=pts["lat"][idx], time=pts["time"][idx],
              accuracy=pts["accuracy"][idx])
    opts = engine.default_options(1) if opts is None else opts
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                               np.zeros(len(wins), np.uint32)))
    return wins, tr, ref


def _oracle_tiles(ref, tr, privacy, quantisation=3600):
    rmask = tmask = engine.levels_mask((0, 1))
    files = {}
    for k in range(len(tr["trace_off"]) - 1):
        s0, s1 = ref["seg_off"][k], ref["seg_off"][k + 1]
        o0, o1 = tr["trace_off"][k], tr["trace_off"][k + 1]
        reps, _ = mo.report_trace(ref["segs"][s0:s1], tr["time"][o1 - 1], 15.0, rmask, tmask)
        rd = [{"id": int(r["id"]), "next_id": int(r["next_id"]), "t0": float(r["t0"]), "t1": float(r["t1"]),
               "length": int(r["length"]), "queue_length": int(r["queue_length"])} for r in reps]
        lines = to.tile_lines(rd, int(tr["time"][o0]), int(tr["time"][o1 - 1]), quantisation, "smpl_rprt", "auto")
        for name, ls in lines.items():
            files.setdefault(name, []).extend(ls)
    out = {}
    for name, ls in files.items():
        body = to.tile_body(ls, privacy)
        if body is not None:
            out[name] = body
    return out


def test_points_windows_match_and_tiles(small_world):
    path = small_world
    g = graphfile.load(path)
    eng = engine.Engine(path, 0)
    pts = _stream(path)
    bm = engine.BatchMatcher(eng)
    bm.run_points(pts["uuid"], pts["time"], pts["lon"], pts["lat"], pts["accuracy"], inactivity=120)
    wins, tr, ref = _oracle(g, pts)
    assert len(wins) == 80
    # windows: same vehicles, same points in the same order
    np.testing.assert_array_equal(bm.trace_uuid(), np.array([u for u, _ in wins], np.uint32))
    gb = bm.batch()
    np.testing.assert_array_equal(gb["trace_off"], tr["trace_off"])
    np.testing.assert_array_equal(gb["time"], tr["time"])
    np.testing.assert_array_equal(gb["lon"], tr["lon"].astype(np.float32))
    np.testing.assert_array_equal(gb["lat"], tr["lat"].astype(np.float32))
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["segments"] > 100
    total = 0
    for privacy in (1, 2, 3):
        got = bm.tiles(privacy=privacy)
        want = _oracle_tiles(ref, tr, privacy)
        assert got == want
        total += len(got)
    assert total > 0


def test_points_with_turn_costs(small_world):
    """run_points checks and applies a batch's options as run() does: with auto's stock turn
    costs (200) every stage equals the oracle at 200, and a negative factor is refused."""
    g = graphfile.load(small_world)
    eng = engine.Engine(small_world, 0)
    pts = _stream(small_world)
    opts = engine.default_options(1, turn_penalty_factor=200.0)
    bm = engine.BatchMatcher(eng)
    bm.run_points(pts["uuid"], pts["time"], pts["lon"], pts["lat"], pts["accuracy"], inactivity=120, opts=opts)
    wins, tr, ref = _oracle(g, pts, opts=opts)
    valid = ref["route"] != 0xffffffff
    assert int((ref["route_turn"][valid] > 0).sum()) > 1000
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["segments"] > 100
    with pytest.raises(RuntimeError, match="turn_penalty_factor"):
        bm.run_points(pts["uuid"], pts["time"], pts["lon"], pts["lat"], pts["accuracy"],
                      opts=engine.default_options(1, turn_penalty_factor=-1.0))
    bm.close()
    eng.close()


def test_tiles_empty_and_errors(small_world):
    eng = engine.Engine(small_world, 0)
    bm = engine.BatchMatcher(eng)
    one = np.array([0], np.uint32)
    bm.run_points(one, np.array([1.5e9]), np.array([8.0]), np.array([47.0]))   # a single point: no window
    assert bm.sizes()["traces"] == 0
    with pytest.raises(RuntimeError):
        bm.run_points(np.array([0, 5], np.uint32), np.array([1.0, 2.0]), np.zeros(2), np.zeros(2), n_uuids=2)


def test_batch_cli_end_to_end(small_world, tmp_path):
    """reporter_amd.batch over trace files in the reference's on-disk format."""
    from reporter_amd import batch
    g = graphfile.load(small_world)
    pts = _stream(small_world, n_veh=24, seed=8)
    tdir = tmp_path / "traces"
    tdir.mkdir()
    for f in range(3):   # points of a vehicle may be spread over files (appends from several downloads)
        sel = np.arange(len(pts["uuid"])) % 3 == f
        with open(tdir / ("%03x" % f), "w") as fh:
            for u, t, la, lo, a in zip(pts["uuid"][sel], pts["time"][sel], pts["lat"][sel], pts["lon"][sel],
                                       pts["accuracy"][sel]):
                fh.write("v%d,%d,%.6f,%.6f,%d\n" % (u, int(t), la, lo, int(a)))
    conf = tmp_path / "conf.json"
    conf.write_text(json.dumps({"meili": {"default": {}}, "reporter_amd": {"graph": small_world}}))
    files = batch.run([str(p) for p in tdir.iterdir()], str(conf), str(tmp_path / "out"), privacy=2)
    # oracle over the same parsed points (file order, dense ids in first-seen order)
    uuids, parsed = batch.read_trace_files(sorted(str(p) for p in tdir.iterdir()))
    idx, _ = batch.dense_ids(uuids)
    op = dict(uuid=idx, time=parsed["time"], lon=parsed["lon"], lat=parsed["lat"], accuracy=parsed["accuracy"])
    _, tr, ref = _oracle(g, op)
    want = _oracle_tiles(ref, tr, 2)
    assert files == want and len(files) > 0
    for name, body in want.items():
        assert (tmp_path / "out" / name).read_text() == body
