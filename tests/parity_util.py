"""Stage-by-stage comparison of the HIP engine against the CPU oracle."""
import numpy as np


def state_slots(trace_off, n_states):
    """Boolean mask of point slots that hold a state layer."""
    P = int(trace_off[-1])
    m = np.zeros(P, bool)
    for k in range(len(trace_off) - 1):
        o = int(trace_off[k])
        m[o:o + int(n_states[k])] = True
    return m


def _ranges(starts, lens):
    """Concatenated index ranges [starts[i], starts[i] + lens[i]) (vectorised)."""
    starts = np.asarray(starts, np.int64)
    lens = np.asarray(lens, np.int64)
    total = int(lens.sum())
    if total == 0:
        return np.zeros(0, np.int64)
    first = np.cumsum(lens) - lens
    return np.repeat(starts - first, lens) + np.arange(total, dtype=np.int64)


def compare_all(gpu, ref, trace_off, check_reports=True):
    """Assert bit-exact agreement of every stage; returns a dict of counts."""
    n_states, orig = gpu.states()
    np.testing.assert_array_equal(n_states, ref["n_states"], "n_states")
    sm = state_slots(trace_off, n_states)
    np.testing.assert_array_equal(orig[sm], ref["state_orig"][sm], "state_orig")

    cn, road, s, sq = gpu.candidates()
    np.testing.assert_array_equal(cn[sm], ref["cand_n"][sm], "cand_n")
    kmask = np.arange(16)[None, :] < cn[:, None]
    kmask &= sm[:, None]
    np.testing.assert_array_equal(road[kmask], ref["cand_road"][kmask], "cand_road")
    np.testing.assert_array_equal(s[kmask], ref["cand_s"][kmask], "cand_s")
    np.testing.assert_array_equal(sq[kmask].view(np.uint32), ref["cand_sq"][kmask].view(np.uint32), "cand_sq bits")

    toff, gc, route = gpu.routes()
    first = np.zeros(len(sm), bool)
    first[trace_off[:-1][n_states > 0]] = True
    tm = sm & ~first
    np.testing.assert_array_equal(toff[tm], ref["trans_off"][tm], "trans_off")
    np.testing.assert_array_equal(gc[tm].view(np.uint64), ref["gc"][tm].view(np.uint64), "gc bits")
    np.testing.assert_array_equal(route, ref["route"], "route_cm")
    # with turn costs (rule 3b) K2 hands K3 every transition's distance term turn_m + |route_m - gc|:
    # bit for bit the oracle's (this checks every turn weight); without them there is none
    d = gpu.route_terms()
    if d is None:
        assert not ref["route_turn"].any(), "the oracle weighs turns the engine did not"
    else:
        np.testing.assert_array_equal(d.view(np.uint64), ref["route_d"].view(np.uint64), "route distance terms")

    choice, cs = gpu.viterbi()
    np.testing.assert_array_equal(cs[sm], ref["chain_start"][sm], "chain_start")
    np.testing.assert_array_equal(choice[sm], ref["choice"][sm], "choice")

    poff, pcnt, pool, rdist = gpu.paths()
    inchain = tm & (cs == 0) & (choice >= 0)
    np.testing.assert_array_equal(pcnt[inchain], ref["path_cnt"][inchain], "path_cnt")
    np.testing.assert_array_equal(rdist[inchain], ref["route_dist"][inchain], "route_dist")
    sel = np.nonzero(inchain)[0]
    lens = pcnt[sel].astype(np.int64)
    a = pool[_ranges(poff[sel], lens)]
    b = ref["path_pool"][_ranges(ref["path_off"][sel], lens)]
    if not np.array_equal(a, b):
        bad = np.nonzero(a != b)[0][0]
        p = sel[np.searchsorted(np.cumsum(lens), bad, side="right")]
        raise AssertionError("path edges differ at slot %d: gpu %s oracle %s" % (
            p, pool[poff[p]:poff[p] + pcnt[p]],
            ref["path_pool"][ref["path_off"][p]:ref["path_off"][p] + ref["path_cnt"][p]]))

    soff, segs = gpu.segments()
    np.testing.assert_array_equal(soff, ref["seg_off"], "seg_off")
    if len(segs):
        for f in segs.dtype.names:
            a, b = segs[f], ref["segs"][f]
            if a.dtype.kind == "f":
                a, b = a.view(np.uint64), b.view(np.uint64)
            np.testing.assert_array_equal(a, b, "segments." + f)
    return dict(points=int(trace_off[-1]), states=int(sm.sum()), transitions=len(route),
                chained=int(inchain.sum()), segments=len(segs))


def _levels_mask(levels):
    from reporter_amd import engine
    return engine.levels_mask(levels)


def check_reports(bm, ref, tr, rl=(0, 1), tl=(0, 1), threshold=15.0):
    """report() per trace: GPU k_report against the oracle's og_report_trace, bit for bit."""
    import meili_oracle as mo
    off, reps, stats = bm.reports()
    rmask, tmask = _levels_mask(rl), _levels_mask(tl)
    T = len(tr["trace_off"]) - 1
    wants, wsts = [], []
    for k in range(T):
        s0, s1 = ref["seg_off"][k], ref["seg_off"][k + 1]
        end_t = tr["time"][tr["trace_off"][k + 1] - 1]
        want, wst = mo.report_trace(ref["segs"][s0:s1], end_t, threshold, rmask, tmask)
        if off[k + 1] - off[k] != len(want):
            raise AssertionError("trace %d: %d reports vs %d" % (k, off[k + 1] - off[k], len(want)))
        wants.append(want)
        wsts.append(wst)
    want = np.concatenate(wants) if wants else reps[:0]
    got = reps[off[0]:off[T]]
    for f in want.dtype.names:
        a, b = got[f], want[f]
        if a.dtype.kind == "f":
            a, b = a.view(np.uint64), b.view(np.uint64)
        np.testing.assert_array_equal(a, b, "report field " + f)
    for f in stats.dtype.names:
        np.testing.assert_array_equal(stats[f][:T].astype(np.int64), np.array([w[f] for w in wsts], np.int64),
                                      "stat " + f)
    return len(got)


def truth_recovery(trace_off, n_states, state_orig, cand_road, choice, truth_edge, edges):
    """Fraction of matched states (choice >= 0) whose chosen road is the road the generator
    drove at that point (world.generate_traces truth_edge): an independent check of the
    matcher's spec that the GPU/oracle bit-parity cannot give (a rule both sides get wrong
    the same way still loses the truth).  Returns (fraction, matched states, all states)."""
    E = np.asarray(edges).reshape(-1, 4)
    truth_road = E[np.asarray(truth_edge, np.int64), 3] >> 1
    trace_off = np.asarray(trace_off, np.int64)
    T = len(trace_off) - 1
    ns = np.asarray(n_states, np.int64)
    slots = _ranges(trace_off[:-1], ns)
    owner = np.repeat(np.arange(T), ns)
    pts = trace_off[owner] + np.asarray(state_orig, np.int64)[slots]
    ch = np.asarray(choice)[slots].astype(np.int64)
    ok = ch >= 0
    chosen = np.asarray(cand_road).reshape(-1, 16)[slots[ok], ch[ok]]
    hit = int((chosen == truth_road[pts[ok]]).sum())
    return hit / max(int(ok.sum()), 1), int(ok.sum()), len(slots)


def match_and_compare(path, tr, opts, trace_opt, rl=(0, 1), tl=(0, 1), hist=False, ball_radius=None, keep_ref=False):
    """Run the engine on a trace set and compare every stage, report() and (hist) the speed
    histogram and duration sums with the oracle; returns compare_all's counts plus tiers."""
    import ctypes

    import meili_oracle as mo
    from reporter_amd import _lib, engine, graphfile
    g = graphfile.load(path)
    eng = engine.Engine(path, 0)
    if ball_radius is not None:
        eng.set_ball_radius(ball_radius)
    T = len(tr["trace_off"]) - 1
    if trace_opt is None:
        trace_opt = np.zeros(T, np.uint32)
    nseg = eng.n_segments
    dptr, uptr = ctypes.c_void_p(), ctypes.c_void_p()
    rp = dict(report_levels=rl, transition_levels=tl)
    if hist:
        _lib.check(_lib.lib().rm_device_alloc(nseg * 16 * 4, ctypes.byref(dptr)))
        _lib.check(_lib.lib().rm_device_alloc(nseg * 8, ctypes.byref(uptr)))
        rp.update(hist_dev=dptr.value, dur_dev=uptr.value, zero_hist=True)
    try:
        bm = engine.BatchMatcher(eng)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt, **rp)
        if hist:
            got_hist = np.empty(nseg * 16, np.uint32)
            _lib.check(_lib.lib().rm_device_download(got_hist.ctypes.data, dptr, got_hist.nbytes))
            got_dur = np.empty(nseg, np.uint64)
            _lib.check(_lib.lib().rm_device_download(got_dur.ctypes.data, uptr, got_dur.nbytes))
    finally:
        if hist:
            _lib.lib().rm_device_free(dptr)
            _lib.lib().rm_device_free(uptr)
    batch = mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    ref = mo.match(g, batch)
    c = compare_all(bm, ref, tr["trace_off"])
    c["reports"] = check_reports(bm, ref, tr, rl=rl, tl=tl)
    if hist:
        want = np.zeros(nseg * 16, np.uint32)
        want_dur = np.zeros(nseg, np.uint64)
        nvalid = mo.pipeline(g, batch, 15.0, engine.levels_mask(rl), engine.levels_mask(tl), want, want_dur)
        np.testing.assert_array_equal(got_hist, want, "speed histogram")
        np.testing.assert_array_equal(got_dur, want_dur, "per-segment duration sums")
        assert int(got_dur.sum()) > 0
        assert int(got_hist.sum()) == nvalid
        c["valid_reports"] = nvalid
    c["traces"] = T
    c["route_tiers"] = bm.route_tiers()
    c["ball_stats"] = eng.ball_stats(0)
    if keep_ref:
        c["_ref"] = ref
    bm.close()
    eng.close()
    return c
