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
