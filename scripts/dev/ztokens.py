"""Token-level view of a raw deflate bit stream (debugging the zlib stage)."""
import sys

LBASE = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LEXT = [0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DBASE = [1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DEXT = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]


class Bits:
    def __init__(self, b):
        self.b, self.pos = b, 0
    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.b[self.pos >> 3] >> (self.pos & 7)) & 1) << i
            self.pos += 1
        return v
    def align(self):
        self.pos = (self.pos + 7) & ~7


def huff(lens):
    code, tab = 0, {}
    bl = [0] * 16
    for l in lens:
        if l: bl[l] += 1
    nxt = [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for s, l in enumerate(lens):
        if l:
            tab[(l, nxt[l])] = s
            nxt[l] += 1
    return tab


def dec(bs, tab):
    code = l = 0
    while True:
        code = (code << 1) | bs.get(1)
        l += 1
        if (l, code) in tab:
            return tab[(l, code)]


def tokens(raw, skip=0):
    bs = Bits(raw)
    bs.pos = skip * 8
    out = []
    while bs.pos < len(raw) * 8 - 7:
        last = bs.get(1); t = bs.get(2)
        blk = {'type': t, 'last': last, 'start_bit': bs.pos - 3, 'toks': []}
        if t == 0:
            bs.align(); L = bs.get(16); bs.get(16)
            blk['stored'] = L; bs.pos += 8 * L
        else:
            if t == 1:
                lt = huff([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8); dt = huff([5] * 30)
            else:
                hl, hd, hc = bs.get(5) + 257, bs.get(5) + 1, bs.get(4) + 4
                order = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
                cl = [0] * 19
                for i in range(hc): cl[order[i]] = bs.get(3)
                ct = huff(cl); lens = []
                while len(lens) < hl + hd:
                    s = dec(bs, ct)
                    if s < 16: lens.append(s)
                    elif s == 16: lens += [lens[-1]] * (3 + bs.get(2))
                    elif s == 17: lens += [0] * (3 + bs.get(3))
                    else: lens += [0] * (11 + bs.get(7))
                lt, dt = huff(lens[:hl]), huff(lens[hl:])
            while True:
                s = dec(bs, lt)
                if s < 256: blk['toks'].append(s)
                elif s == 256: break
                else:
                    c = s - 257; ln = LBASE[c] + bs.get(LEXT[c])
                    d = dec(bs, dt); dist = DBASE[d] + bs.get(DEXT[d])
                    blk['toks'].append((ln, dist))
        out.append(blk)
        if last or (t == 0 and blk.get('stored') == 0): break
    return out
