"""Bank model of csrc/gemm_tn.hip's transposed fragment reads (ds_read_b64_tr_b16: two 32-lane groups, 64 x 4-byte
banks each): for every chunk count per token row (CPA = BM / 8), find a row rotation rot(t) of the 16-byte chunks such
that every 32-lane half of every fragment read (token rows 32 ks + 8 h + q (+4), h in {0, 1} or {2, 3}, q = 0..3; the
two chunks of a 16-column block) touches 16 distinct 16-byte bank slots. Prints the (x1, x2, x3) of
rot(t) = x1 (t & 3) + x2 ((t >> 2) & 1) + x3 ((t >> 3) & 3) mod CPA that the kernel uses."""
import itertools
def ok(CPA, rot, xor=False):
    for ks in (0,1):
        for second in (0,1):
            for half in (0,1):
                rows=[32*ks+8*h+q+4*second for h in ((0,1) if half==0 else (2,3)) for q in range(4)]
                for c0 in range(0, CPA-1, 2):
                    slots=set()
                    for t in rows:
                        for c in (c0,c0+1):
                            cp = (c ^ rot(t)) if xor else (c+rot(t))%CPA
                            slots.add((t*CPA+cp)%16)
                    if len(slots)<16: return False
    return True
for CPA in (6, 8, 12, 16, 24):
    found=None
    for x1,x2,x3 in itertools.product(range(CPA),repeat=3):
        rot=lambda t: (x1*(t&3)+x2*((t>>2)&1)+x3*((t>>3)&3))
        if ok(CPA, lambda t: rot(t)%CPA):
            found=('add',x1,x2,x3); break
    if found is None and CPA in (8,16):
        for x1,x2,x3 in itertools.product(range(CPA),repeat=3):
            rot=lambda t: (x1*(t&3)^x2*((t>>2)&1)^x3*((t>>3)&3))%CPA
            if ok(CPA, rot, True):
                found=('xor',x1,x2,x3); break
    print(CPA, found)
