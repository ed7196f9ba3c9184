"""LDS bank model of csrc/attention.hip short kernels (S <= 128): cycles per instruction relative to conflict-free, per
access site, for candidate row lengths LD (K / V / Q / dO images) and LP (P_d / dS staging). Bank rules:
MI355X_MICROARCH.md LDS table (tools/lds_banks.py). Run from the repo root: python tools/lds_banks_attn.py"""
import sys
sys.path.insert(0, "tools")
from lds_banks import cycles, GROUPS

def site_stats(LD, LP, S=128):
    res = {}
    # scores (fwd & bwd): ds_read_b128 at (16kt + r)*LD + 32ks + 8h
    c = []
    for kt in range(S//16):
        for ks in range(2):
            a = [2*((16*kt + (l&15))*LD + 32*ks + 8*(l>>4)) for l in range(64)]
            c.append(cycles(a, "b128"))
    res["scores_b128"] = sum(c)/len(c)/4
    # O^T / dQ^T: tr_read at (32ks + 4h + q)*LD + 16dt + 4p and +16*LD
    c = []
    for ks in range(S//32):
        for dt in range(4):
            for off in (0, 16):
                a = []
                for l in range(64):
                    r, h = l & 15, l >> 4
                    q, p = r >> 2, r & 3
                    a.append(2*((32*ks + 4*h + q + off)*LD + 16*dt + 4*p))
                c.append(cycles(a, "b64"))
    res["vT_tr"] = sum(c)/len(c)/2
    # load_rows: ds_write_b128 row*LD + ch*8, c = tid
    c = []
    for base in range(0, S*8, 64):
        a = [2*(((base + l) >> 3)*LD + ((base + l) & 7)*8) for l in range(64)]
        c.append(cycles(a, "w128"))
    res["load_w128"] = sum(c)/len(c)/8
    # bwd: P_d / dS staging write ds_write_b64 at qi*LP + 16kt + 4h, qi = 16w + r
    c = []
    for w in range(S//16):
        for kt in range(S//16):
            a = [2*((16*w + (l&15))*LP + 16*kt + 4*(l>>4)) for l in range(64)]
            c.append(cycles(a, "w64"))
    res["stage_w64"] = sum(c)/len(c)/4
    # bwd dV/dK: tr_read dOs/Qs at row*LD + 16dt + 4p (+4*LD), row = 32s + 8h + q
    c = []; c2 = []
    for s in range(S//32):
        for dt in range(4):
            for off in (0, 4):
                a = []; b = []
                for l in range(64):
                    r, h = l & 15, l >> 4
                    q, p = r >> 2, r & 3
                    row = 32*s + 8*h + q + off
                    a.append(2*(row*LD + 16*dt + 4*p))
                    b.append(2*(row*LP + 16*0 + 4*p))  # kj = 16w: take w=0
                c.append(cycles(a, "b64")); c2.append(cycles(b, "b64"))
    res["bwd_tr_LD"] = sum(c)/len(c)/2
    res["bwd_tr_LP"] = sum(c2)/len(c2)/2
    return res

for LD in (72, 80, 88, 96, 104, 136):
    for LP in (136, 144, 152, 160, 168):
        r = site_stats(LD, LP)
        print(LD, LP, {k: round(v, 2) for k, v in r.items()})

print("---- with row perm (bit3 -> bit2 xor) on the staged images")
def perm(row):
    return row ^ (((row >> 3) & 1) << 2)
def bwd_sites(LD, LP, S=128, pm=perm):
    res = {}
    c = []; c2 = []
    for s in range(S//32):
        for dt in range(4):
            for off in (0, 4):
                a = []; b = []
                for l in range(64):
                    r, h = l & 15, l >> 4
                    q, p = r >> 2, r & 3
                    row = 32*s + 8*h + q + off
                    a.append(2*(pm(row)*LD + 16*dt + 4*p))
                    b.append(2*(pm(row)*LP + 16*0 + 4*p))
                c.append(cycles(a, "b64")); c2.append(cycles(b, "b64"))
    res["bwd_tr_LD"] = sum(c)/len(c)/2
    res["bwd_tr_LP"] = sum(c2)/len(c2)/2
    c = []
    for w in range(S//16):
        for kt in range(S//16):
            a = [2*(pm(16*w + (l&15))*LP + 16*kt + 4*(l>>4)) for l in range(64)]
            c.append(cycles(a, "w64"))
    res["stage_w64"] = sum(c)/len(c)/4
    # Qs/dOs b128 row reads at qi = 16w + r (perm applied)
    c = []
    for w in range(S//16):
        for ks in range(2):
            a = [2*(pm(16*w + (l&15))*LD + 32*ks + 8*(l>>4)) for l in range(64)]
            c.append(cycles(a, "b128"))
    res["q_b128"] = sum(c)/len(c)/4
    c = []
    for base in range(0, S*8, 64):
        a = [2*(pm((base + l) >> 3)*LD + ((base + l) & 7)*8) for l in range(64)]
        c.append(cycles(a, "w128"))
    res["load_w128"] = sum(c)/len(c)/8
    return res
for LD in (72, 80):
    for LP in range(128, 200, 8):
        print(LD, LP, {k: round(v, 2) for k, v in bwd_sites(LD, LP).items()})

print("---- granule XOR swizzle on Q/dO images, LD=80")
def qsites(LD, swz, S=128):
    def addr(row, col):
        g, e = divmod(col, 4)
        g = g ^ swz(row)
        return 2*(row*LD + 4*g + e)
    res = {}
    c = []
    for s in range(S//32):
        for dt in range(4):
            for off in (0, 4):
                a = []
                for l in range(64):
                    r, h = l & 15, l >> 4
                    q, p = r >> 2, r & 3
                    row = 32*s + 8*h + q + off
                    a.append(addr(row, 16*dt + 4*p))
                c.append(cycles(a, "b64"))
    res["tr"] = sum(c)/len(c)/2
    c = []
    for w in range(S//16):
        for ks in range(2):
            a = [addr(16*w + (l&15), 32*ks + 8*(l>>4)) for l in range(64)]
            c.append(cycles(a, "b128"))
    res["b128"] = sum(c)/len(c)/4
    c = []
    for base in range(0, S*8, 64):
        a = [addr((base + l) >> 3, ((base + l) & 7)*8) for l in range(64)]
        c.append(cycles(a, "w128"))
    res["w128"] = sum(c)/len(c)/8
    return res
best = []
for cbit in range(0, 5):
    for c in range(0, 16, 2):
        swz = lambda row, cbit=cbit, c=c: c * ((row >> cbit) & 1)
        r = qsites(80, swz)
        best.append((r["tr"] + r["b128"] + r["w128"], cbit, c, r))
best.sort(key=lambda x: x[0])
for b in best[:6]:
    print(b)
