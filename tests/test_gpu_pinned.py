"""What can be pinned beyond GPU-vs-oracle parity (GPU).

1. The device report() epilogue against the reference's OWN outputs: all 415 cases of
   tests/golden/report_golden.json (produced by running reference
   py/reporter_service.py:79-179, see tests/golden/make_report_golden.py) go through
   rm_report_segments — shapes the matcher never produces (missing ``internal`` keys,
   negative dt, t0 = -1 priors, empty lists, thresholds 0/5/60, level sets [] / [2]).
2. Truth recovery: the generator knows the road it drove at every point
   (world.generate_traces truth_edge).  A rule the GPU and the oracle got wrong the same
   way keeps bit-parity but loses the truth, so each config's recovery rate is asserted
   on the GPU's own choices, with thresholds measured on the oracle.
"""
import json
import os

import numpy as np
import pytest

import meili_oracle as mo
from parity_util import compare_all, truth_recovery
from reporter_amd import engine, graphfile, world
from test_report_oracle import _to_records

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "report_golden.json")


def test_device_report_matches_reference_goldens(built_lib):
    with open(GOLDEN) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == 415
    segs = [_to_records(c["input"]["match"]["segments"]) for c in cases]
    seg_off = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.uint32)
    allsegs = np.concatenate(segs) if len(seg_off) > 1 else segs[0]
    inp = [c["input"] for c in cases]
    rep_off, reps, stats = engine.report_segments(
        seg_off, allsegs, [c["trace_end_time"] for c in inp], [c["threshold_sec"] for c in inp],
        [engine.levels_mask(c["report_levels"]) for c in inp], [engine.levels_mask(c["transition_levels"]) for c in inp])
    km = lambda m: 0 if m < 0 else round(m * 0.001, 3)
    n_rep = 0
    for i, rec in enumerate(cases):
        want = rec["output"]
        got = reps[rep_off[i]:rep_off[i + 1]]
        wr = want["datastore"]["reports"]
        assert len(got) == len(wr), "case %d" % i
        for r, w in zip(got, wr):
            assert int(r["id"]) == w["id"] and float(r["t0"]) == w["t0"] and float(r["t1"]) == w["t1"], i
            assert int(r["length"]) == w["length"] and int(r["queue_length"]) == w["queue_length"], i
            assert (int(r["next_id"]) if int(r["next_id"]) != engine.INVALID_SEGMENT_ID else None) == w.get("next_id"), i
        st, ws = stats[i], want["stats"]
        assert int(st["successful_count"]) == ws["successful_matches"]["count"], i
        assert int(st["unreported_count"]) == ws["unreported_matches"]["count"], i
        assert km(int(st["successful_length_m"])) == ws["successful_matches"]["length"], i
        assert km(int(st["unreported_length_m"])) == ws["unreported_matches"]["length"], i
        assert int(st["discontinuities"]) == ws["match_errors"]["discontinuities"], i
        assert int(st["invalid_speeds"]) == ws["match_errors"]["invalid_speeds"], i
        assert int(st["invalid_times"]) == ws["match_errors"]["invalid_times"], i
        assert int(st["unassociated"]) == ws["unassociated_segments"], i
        assert (int(st["shape_used"]) if st["shape_used"] >= 0 else None) == want.get("shape_used"), i
        n_rep += len(got)
    assert n_rep > 150   # 175 reports across the 415 reference outputs


def _world(tmpdir_session, name):
    cfg = dict(world.CONFIGS[name])
    path = str(tmpdir_session / ("truth_%s.rmg" % name))
    if not os.path.exists(path):
        world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    return path, cfg


def _gpu_recovery(path, tr, opts, trace_opt):
    g = graphfile.load(path)
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt))
    compare_all(bm, ref, tr["trace_off"])
    n_states, orig = bm.states()
    _, road, _, _ = bm.candidates()
    choice, _ = bm.viterbi()
    out = {}
    for q in np.unique(trace_opt):
        ks = np.nonzero(trace_opt == q)[0]
        o = tr["trace_off"]
        sel_off = np.concatenate([[0], np.cumsum([o[k + 1] - o[k] for k in ks])])
        pts = np.concatenate([np.arange(o[k], o[k + 1]) for k in ks])
        # the helper indexes slots from trace_off: rebase every array onto the selected traces
        r = truth_recovery(sel_off, n_states[ks], orig[pts], road[pts], choice[pts], tr["truth_edge"][pts], g["edges"])
        out[int(q)] = r
    bm.close()
    eng.close()
    return out


@pytest.mark.parametrize("name,n_traces,floor", [("C2", 300, 0.93), ("C3", 1500, 0.95)])
def test_truth_recovery_c2_c3(built_lib, tmpdir_session, name, n_traces, floor):
    """C2 (1 Hz urban) and C3 (30 s sampling, 100 m radius, kilometre routes): the road the
    GPU picks is the road driven (oracle on the same inputs: C2 0.946, C3 0.964)."""
    path, cfg = _world(tmpdir_session, name)
    tr = world.generate_traces(path, n_traces, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=1000)
    opts = engine.default_options(1, search_radius=cfg["search_radius"])
    frac, n, _ = _gpu_recovery(path, tr, opts, np.zeros(n_traces, np.uint32))[0]
    print(name, "truth recovery", frac, n)
    assert n > 50_000 and frac >= floor, (frac, n)


# oracle rates on these inputs (100 traces each): auto .978/.957/.915/.838, bicycle
# .981/.964/.930/.823, pedestrian .982/.964/.921/.783 for sigma_z 2/4.07/8/16
C5_FLOORS = {2.0: 0.96, 4.07: 0.94, 8.0: 0.89, 16.0: 0.75}


def test_truth_recovery_c5_modes_sigma(built_lib, tmpdir_session):
    path, cfg = _world(tmpdir_session, "C2")
    parts, opts, keys = [], [], []
    for mode in ("auto", "bicycle", "pedestrian"):
        for sz in sorted(C5_FLOORS):
            parts.append(world.generate_traces(path, 100, 600, 1.0, sz, seed=5000, mode=mode))
            opts.append(engine.default_options(1, mode=world.MODES[mode], sigma_z=sz, search_radius=max(50.0, 3 * sz))[0])
            keys.append((mode, sz))
    tr = {k: np.concatenate([p[k] for p in parts]) for k in ("lon", "lat", "time", "accuracy", "truth_edge")}
    tr["trace_off"] = (np.arange(len(parts) * 100 + 1) * 600).astype(np.uint32)
    trace_opt = np.repeat(np.arange(len(parts), dtype=np.uint32), 100)
    res = _gpu_recovery(path, tr, np.array(opts, engine.OPTIONS_DTYPE), trace_opt)
    for q, (mode, sz) in enumerate(keys):
        frac, n, _ = res[q]
        print("C5", mode, sz, "truth recovery", round(frac, 4), n)
        assert n > 5000 and frac >= C5_FLOORS[sz], (mode, sz, frac)
