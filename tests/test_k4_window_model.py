"""The K4 window algebra against the oracle's segments (CPU).

`k_seg_wave` (reporter_amd/csrc/engine.hip) forms a trace's segments 64 traversal records at a
time, one record per lane, with meili's form_segments rules rewritten as mask algebra over
ballots and segmented prefix sums, and carries the open run / piece across windows.  This is a
lane-by-lane Python model of exactly that algebra (same masks, same carries), run on the
oracle's own paths and compared with the oracle's sequential segment forming
(oracle/meili_oracle.c og_segments) — so the window decomposition itself is checked on CPU, for
every travel mode and for sparse sampling with long and broken chains.  The GPU kernel is then
checked bit for bit against the oracle by the -m gpu parity tests.
"""
import numpy as np
import pytest

import meili_oracle as mo
from reporter_amd import engine, graphfile, world

NONE = 0xffffffff
LAST, INTF = 1 << 30, 1 << 31
MASK = LAST - 1
V_QUEUE = 2.7777777777777777  # 10 km/h in m/s (engine.hip kQueueSpeedMps)
FLAG_INTERNAL = 1 << 19       # EdgeRec::info bit (rm_common.hpp)


def same_chain(a, b):
    return b == a or b == ((a + 1) & 0xffffffff)


def interp(ta, tb, x, d):
    return ta if d == 0 else ta + (tb - ta) * (float(x) / float(d))


def hi_le(m, i):   # highest set bit <= i, or -1
    if i < 0:
        return -1
    mm = m & ((2 << i) - 1)
    return mm.bit_length() - 1 if mm else -1


def lo_gt(m, i):   # lowest set bit > i, or 64
    mm = m & ~((2 << i) - 1) & ((1 << 64) - 1)
    return (mm & -mm).bit_length() - 1 if mm else 64


def flag_vs(t, has, u):   # engine.hip flag_vs: (kind 1 new / 2 merged, head)
    if not has:
        return 1, 1
    if u["e"] == t["e"] and u["en"] == t["b"]:
        return 2, 0
    cont = u["sd"] == t["sd"]
    if cont and t["sd"] == NONE and ((u["slot"] ^ t["slot"]) & INTF):
        cont = False
    if cont:
        if u["en"] != u["len"] or t["b"] != 0:
            cont = False
        elif t["sd"] != NONE and t["soff"] != u["soff"] + u["len"]:
            cont = False
    return 1, 0 if cont else 1


def slow(md, mtb, mte):
    dt = mte - mtb
    return dt > 0.0 and (float(md) * 0.01) / dt < V_QUEUE


def bits(flags):
    return sum(1 << i for i, f in enumerate(flags) if f)


def model_segments(g, tr, ref):
    """Segments per trace as k_seg_wave forms them (start/end time, length, queue, ways)."""
    E = g["edges"].reshape(-1, 4)
    P, T = len(tr["lon"]), len(tr["trace_off"]) - 1
    toff, so, ns_, choice, cs = tr["trace_off"], ref["state_orig"], ref["n_states"], ref["choice"], ref["chain_start"]
    valid = np.zeros(P, bool)
    st_time = np.zeros(P)
    for k in range(T):
        o = toff[k]
        for s in range(ns_[k]):
            st_time[o + s] = tr["time"][o + so[o + s]]
            if s and cs[o + s] == 0 and choice[o + s] >= 0 and choice[o + s - 1] >= 0:
                valid[o + s] = True
    pc = np.where(valid, ref["path_cnt"], 0).astype(np.int64)
    trav = np.concatenate([[0], np.cumsum(pc)[:-1]])
    total = int(pc.sum())
    rec_slot = np.repeat(np.arange(P), pc)
    out_all = []
    for k in range(T):
        o, o1 = int(toff[k]), int(toff[k + 1])
        Rb = int(trav[o]) if o < P else total
        Re = int(trav[o1]) if o1 < P else total
        c_slot, c_has, lk = NONE, False, None
        r_open, r, p_md, p_mtb, carry_x, runs, out = False, {}, 0, 0.0, 0, 0, {}
        c0 = Rb
        while c0 < Re:
            n = min(64, Re - c0)
            last = c0 + n == Re
            recs = []
            for lane in range(64):
                if lane >= n:
                    recs.append(dict(act=False, l=0, q=0, e=0, b=0, en=0, len=0, sd=NONE, soff=0, way=0, slot=0,
                                     ta=0.0, tbs=0.0, D=0))
                    continue
                rr = c0 + lane
                l = int(rec_slot[rr])
                q, ns = rr - int(trav[l]), int(pc[l])
                e = int(ref["path_pool"][ref["path_off"][l] + q])
                L, rev = int(E[e, 1]), int(E[e, 3]) & 1
                sa, sb = int(ref["cand_s"][l - 1][choice[l - 1]]), int(ref["cand_s"][l][choice[l]])
                b0, b1 = 0, L
                if q == 0:
                    b0 = L - sa if rev else sa
                if q + 1 == ns:
                    b1 = L - sb if rev else sb
                slot = l | (LAST if q + 1 == ns else 0) | (INTF if int(E[e, 2]) & FLAG_INTERNAL else 0)
                recs.append(dict(act=True, l=l, q=q, e=e, b=b0, en=b1, len=L, sd=int(g["edge_seg"][e]),
                                 soff=int(g["edge_seg_off"][e]), way=int(g["edge_way"][e]), slot=slot,
                                 ta=st_time[l - 1], tbs=st_time[l], D=int(ref["route_dist"][l])))
            w = [(x["en"] - x["b"]) & 0xffffffff for x in recs]
            S = [int(v) for v in np.cumsum(w)]
            for lane, x in enumerate(recs):   # distance into the transition's route
                st = lane - x["q"]
                xb = S[lane] - w[lane] - (S[st - 1] if st > 0 else 0) + (carry_x if st < 0 else 0)
                x["xb"], x["tb"] = xb, interp(x["ta"], x["tbs"], xb, x["D"])
                x["te"] = interp(x["ta"], x["tbs"], xb + w[lane], x["D"])
            kept = [x["act"] and x["en"] != x["b"] for x in recs]
            K = bits(kept)
            brk = [x["act"] and (not (c_slot != NONE and same_chain(c_slot, x["l"])) if i == 0
                                 else not same_chain(recs[i - 1]["l"], x["l"])) for i, x in enumerate(recs)]
            BR = bits(brk)
            kind, head = [0] * 64, [0] * 64
            for i, x in enumerate(recs):
                if kept[i]:
                    j, pb = hi_le(K, i - 1), hi_le(BR, i)
                    has = pb <= j if j >= 0 else (pb < 0 and c_has)
                    kind[i], head[i] = flag_vs(x, has, recs[j] if j >= 0 else lk)
            NW = bits(kept[i] and kind[i] == 1 for i in range(64))
            HD = bits(kept[i] and head[i] for i in range(64))
            if r_open and K:   # a piece carried in closes before a new piece of its run
                fk = (K & -K).bit_length() - 1
                if (NW >> fk) & 1 and not (HD >> fk) & 1:
                    r["q"] = r["q"] + p_md if slow(p_md, p_mtb, lk["te"]) else 0
            ps = [hi_le(NW, i) for i in range(64)]
            rs = [hi_le(HD, i) for i in range(64)]
            md = [S[i] - (S[ps[i] - 1] if ps[i] > 0 else 0) if ps[i] >= 0 else p_md + S[i] for i in range(64)]
            mtb = [recs[ps[i]]["tb"] if ps[i] >= 0 else p_mtb for i in range(64)]
            nx = [lo_gt(K, i) for i in range(64)]
            closeP = [kept[i] and ((nx[i] < 64 and (NW >> nx[i]) & 1) or (nx[i] == 64 and last)) for i in range(64)]
            endR = [kept[i] and ((nx[i] < 64 and (HD >> nx[i]) & 1) or (nx[i] == 64 and last)) for i in range(64)]
            sl = [closeP[i] and slow(md[i], mtb[i], recs[i]["te"]) for i in range(64)]
            CN = bits(closeP[i] and not sl[i] for i in range(64))
            Qs = [int(v) for v in np.cumsum([md[i] if closeP[i] and sl[i] else 0 for i in range(64)])]
            wf = [recs[rs[i]]["way"] if rs[i] >= 0 else r.get("wf", 0) for i in range(64)]
            MW = bits(kept[i] and kind[i] == 1 and not head[i] and recs[i]["way"] != wf[i] for i in range(64))
            qv, totv, wl = [0] * 64, [0] * 64, [0] * 64
            for i in range(64):
                z, z2 = hi_le(CN, i), hi_le(MW, i)
                if z >= 0 and z >= rs[i]:
                    qv[i] = Qs[i] - Qs[z]
                elif rs[i] >= 0:
                    qv[i] = Qs[i] - (Qs[rs[i] - 1] if rs[i] > 0 else 0)
                else:
                    qv[i] = r.get("q", 0) + Qs[i]
                totv[i] = S[i] - (S[rs[i] - 1] if rs[i] > 0 else 0) if rs[i] >= 0 else r.get("tot", 0) + S[i]
                wl[i] = recs[z2]["way"] if (z2 >= 0 and z2 > rs[i]) else (wf[i] if rs[i] >= 0 else r.get("wl", 0))

            def emit(idx, f, wfv, wlv, tot, q, lst):
                sd = f["sd"]
                seg_len = int(g["seg_len_cm"][sd]) if sd != NONE else 0
                start_ok = f["b"] == 0 and (sd == NONE or f["soff"] == 0)
                end_ok = lst["en"] == lst["len"] and (sd == NONE or lst["soff"] + lst["len"] == seg_len)
                length = ((seg_len + 50) // 100 if start_ok and end_ok else -1) if sd != NONE else (tot + 50) // 100
                out[idx] = (f["tb"] if start_ok else -1.0, lst["te"] if end_ok else -1.0, length, (q + 50) // 100,
                            wfv, wlv)

            if r_open and ((K and (HD >> ((K & -K).bit_length() - 1)) & 1) or (not K and last)):
                emit(r["idx"], r["f"], r["wf"], r["wl"], r["tot"],
                     r["q"] + p_md if slow(p_md, p_mtb, lk["te"]) else 0, lk)
                r_open = False
            for i in range(64):
                if endR[i]:
                    idx = runs + bin(HD & ((2 << i) - 1)).count("1") - 1 if rs[i] >= 0 else r["idx"]
                    emit(idx, recs[rs[i]] if rs[i] >= 0 else r["f"], wf[i], wl[i], totv[i], qv[i], recs[i])
            runs += bin(HD).count("1")
            if last:
                break
            if K:
                jl = K.bit_length() - 1
                if rs[jl] >= 0:
                    r = dict(f=recs[rs[jl]], wf=recs[rs[jl]]["way"], idx=runs - 1)
                r_open = True
                r.update(tot=totv[jl], q=qv[jl], wl=wl[jl])
                p_md, p_mtb, lk = md[jl], mtb[jl], recs[jl]
                c_has = True if jl == 63 else (BR >> (jl + 1)) == 0
            else:
                c_has = c_has and BR == 0
            c_slot, carry_x = recs[n - 1]["l"], recs[n - 1]["xb"] + w[n - 1]
            c0 += 64
        out_all.append([out[i] for i in range(runs)])
    return out_all


@pytest.fixture(scope="module")
def grid(built_lib, tmpdir_session):
    path = str(tmpdir_session / "k4_model.rmg")
    world.build_world(path, 40, 40, 100.0, seed=1, cell_m=100.0)
    return path


@pytest.mark.parametrize("mode,rate,n_pts", [("auto", 1.0, 600), ("bicycle", 1.0, 600), ("pedestrian", 1.0, 600),
                                             ("auto", 30.0, 80), ("auto", 120.0, 40)])
def test_window_algebra_equals_sequential_segments(grid, mode, rate, n_pts):
    g = graphfile.load(grid)
    T = 30
    tr = world.generate_traces(grid, T, n_pts, rate, 5.0, seed=7, mode=mode)
    opts = engine.default_options(1, mode=world.MODES[mode])
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                               np.zeros(T, np.uint32)))
    got = model_segments(g, tr, ref)
    n = 0
    for k in range(T):
        want = ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]]
        assert len(got[k]) == len(want), k
        for a, s in zip(got[k], want):
            assert a == (s["start_time"], s["end_time"], s["length"], s["queue_length"], s["way_first"],
                         s["way_last"]), (k, a, s)
            n += 1
    assert n > 30
