"""The chain fixture (tests/chain_case.py) really is a chain under the oracle
(pinned to the reference): every chunk k >= 1 REFs the previous chunk's block
at offset 1 and then declares its own."""
from chain_case import chain


def test_chain_is_a_chain(oracle):
    d, offs, lens = chain(48)
    outs = oracle.encode_batch(d, offs, lens, mode=1)
    for k in range(1, 48):
        o = outs[k]
        # escape of z (1 or 2 bytes), REF (10 bytes), EXTRACT of E_k (2 + 2048)
        assert len(o) in (1 + 10 + 2050, 2 + 10 + 2050), (k, len(o))
        assert o[-2050:-2048] == b'\xf1\x01' and o[-2048:] == d[int(offs[k]) + 2049:int(offs[k]) + 4097]
        assert o[-2060:-2058] == b'\xf1\x02'
    # the same chunks one at a time from an empty cache: two EXTRACTs (the
    # tiling) and one escaped byte, no REF
    solo = [oracle.encode_batch(d, offs[k:k + 1], lens[k:k + 1], mode=1)[0] for k in range(1, 8)]
    assert all(len(s) in (2 * 2050 + 1, 2 * 2050 + 2) and s[:2] == b'\xf1\x01' and s[2050:2052] == b'\xf1\x01'
               for s in solo)
