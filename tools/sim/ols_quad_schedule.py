"""CPU model of the lab kernel fir_ols_quad_kernel's schedule (kern_fir_ols_os.hip, SDSP_OLS_LAB):
stages, the per-eighth queue counter and the per-tick bookkeeping, with the workgroups' ticks
interleaved at random.  Every segment of an eighth must be loaded, transformed and stored exactly
once, by one slot, with its own data; every index used with a live descriptor lies in [0, cnt);
every workgroup ends within its tick cap.  (Written after the first GPU run of the kernel faulted:
the slot's first S3 read an index that no S2 had published yet.)

    python tools/sim/ols_quad_schedule.py
"""
import random, sys
def run(cnt, J, NS=4, seed=0):
    rnd = random.Random(seed)
    ctr = [0]
    class WG: pass
    wgs = []
    for jb in range(J):
        w = WG(); w.jb = jb
        w.cur = [cnt]*NS; w.nxt = [NS*jb+s if NS*jb+s < cnt else cnt for s in range(NS)]
        w.ph = [2 if s == 0 else -1 for s in range(NS)]
        w.nidx = [-12345]*NS  # LDS garbage: never read before the slot publishes
        w.vn = [None]*NS; w.data = [None]*NS; w.got = [0]*NS
        w.tick = 0; w.go = True; w.cap = 4*cnt+32
        wgs.append(w)
    stored = {}
    loaded = {}
    def valid(k): return 0 <= k < cnt
    while any(w.go for w in wgs):
        w = rnd.choice([w for w in wgs if w.go])
        # one tick of this workgroup: every slot runs its stage
        for s in range(NS):
            ph = w.ph[s]
            if ph == 2:  # S2: queue fetch for the segment after nxt, then the loads of nxt
                if w.nxt[s] < cnt:
                    w.got[s] = ctr[0]; ctr[0] += 1
                k = w.nxt[s]
                w.vn[s] = k if valid(k) else None
                if valid(k): loaded[k] = loaded.get(k, 0) + 1
            elif ph == 3:  # S3: publish the index; P5 and the stores of cur
                g = w.got[s]
                w.nidx[s] = min(cnt, NS*J + g) if (w.nxt[s] < cnt and g < cnt) else cnt
                k = w.cur[s]
                if valid(k):
                    assert w.data[s] == k, ("data mismatch", k, w.data[s])
                    stored[k] = stored.get(k, 0) + 1
            elif ph == 0:  # S0: P1 on the landed loads
                w.data[s] = w.vn[s]
        # end_tick
        live = False
        for s in range(NS):
            if w.ph[s] == 3:
                w.cur[s] = w.nxt[s]
                assert w.nxt[s] >= cnt or w.nidx[s] != -12345, "read before publish"
                w.nxt[s] = w.nidx[s] if w.nxt[s] < cnt else cnt
            w.ph[s] = (2 if w.tick + 1 == s else -1) if w.ph[s] < 0 else (0 if w.ph[s] == 3 else w.ph[s] + 1)
            live = live or w.ph[s] < 0 or w.cur[s] < cnt or w.nxt[s] < cnt
        w.tick += 1
        w.go = live and w.tick < w.cap
    missing = [k for k in range(cnt) if stored.get(k) != 1 or loaded.get(k) != 1]
    assert not missing, ("missing/dup", missing[:10], cnt, J)
    assert all(w.tick < w.cap for w in wgs)
    return max(w.tick for w in wgs)
for cnt in [0, 1, 2, 3, 5, 7, 31, 64, 127, 128, 129, 255, 256, 1000, 4661, 34953]:
    for J in [1, 2, 3, 32]:
        for seed in range(3):
            run(cnt, J, seed=seed)
print("quad schedule ok")
