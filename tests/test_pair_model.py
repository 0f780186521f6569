"""The pair replay's data-parallel formulation (tests/pair_model.py, the one
wanproxy_amd/csrc/xcg_pair.hip computes on the GPU) against a sequential
replay of XCodecCachePair's policy on random reference sequences: primary
hits, disk appends and the write clock, the first inconsistent lookup, the
time every cached entity leaves both levels, and the final LRU order."""
import random

import pytest

from pair_model import ENTER, GMISS, LOOKUP, SeqPair, par_replay


def _scenario(rng):
    C = rng.randint(1, 8)
    ent = rng.randint(2, 4)
    nb = rng.randint(3, 6)
    D = nb * ent
    # warm-up from empty: a consistent starting state
    s = SeqPair(C, nb, ent, [], {}, 0)
    nxt_id = 0
    for j in range(rng.randint(0, 40)):
        live = [x for x in range(nxt_id) if s.present(x)]
        if live and rng.random() < 0.5:
            s.lookup(rng.choice(live), j, j)
        else:
            s.p_enter(nxt_id, j)
            s.d_append(nxt_id, j, j)
            nxt_id += 1
    prim, dent, clock0 = list(s.prim), dict(s.dent), s.clock
    initial = set(prim) | set(dent)
    # the batch: mostly consistent rows (a shadow replay picks present entities)
    shadow = SeqPair(C, nb, ent, prim, dent, clock0)
    rows = []
    lap = D - 2 * ent
    new = []
    for j in range(rng.randint(1, 30)):
        if len(shadow.appends) >= lap - 1:
            break
        r = rng.random()
        live = [x for x in list(initial) + new if shadow.present(x)]
        dead = [x for x in initial if not shadow.present(x)]
        if r < 0.35 or not live:
            x = nxt_id
            nxt_id += 1
            new.append(x)
            rows.append((ENTER, x, j))
            shadow.p_enter(x, j)
            shadow.d_append(x, j, j)
        elif r < 0.85:
            x = rng.choice(live)
            rows.append((LOOKUP, x, j))
            shadow.lookup(x, j, j)
        elif r < 0.95 and dead:
            rows.append((GMISS, rng.choice(dead), j))
        elif initial:   # an inconsistent row: a lookup the parse got wrong
            x = rng.choice(sorted(initial))
            rows.append((LOOKUP if not shadow.present(x) else GMISS, x, j))
            if shadow.present(x):
                shadow.lookup(x, j, j)
    return C, nb, ent, prim, dent, clock0, rows


@pytest.mark.parametrize('seed', range(400))
def test_parallel_replay_equals_sequential(seed):
    rng = random.Random(seed)
    C, nb, ent, prim, dent, clock0, rows = _scenario(rng)
    seq = SeqPair(C, nb, ent, prim, dent, clock0)
    bad = seq.replay(rows)
    lap = nb * ent - 2 * ent
    if len(seq.appends) > lap:
        pytest.skip('sub-batch longer than a disk lap (the engine halves it)')
    par = par_replay(C, nb, ent, prim, dent, clock0, rows)
    assert par['first_bad'] == bad
    if bad is None:
        assert par['final_lru'] == list(seq.prim)
        assert par['appends'] == seq.appends
        assert par['clock'] == seq.clock
        assert par['leave'] == {x: t for x, t in seq.leave.items() if x in set(prim) | set(dent)}
    else:
        tb = rows[bad][2]
        want = {x: t for x, t in seq.leave.items() if t < tb and x in set(prim) | set(dent)}
        got = {x: t for x, t in par['leave'].items() if t < tb}
        assert got == want
        # every entity present at the first bad row stays visible up to it
        for x in set(prim) | set(dent):
            if x not in want:
                assert par['leave'].get(x, 1 << 62) >= tb
