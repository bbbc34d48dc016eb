# Fixed-point round counts of the two-bucket window (np_sampler.hip fast_window) from two
# starting masks, on random words and C2-range states (profiles/r04_np_ab2/r04d_g.txt).
import numpy as np
rng=np.random.default_rng(1)
n1=1999
def run(init, trials=20000):
    it_hist=[]
    for _ in range(trials):
        i=int(rng.integers(200, n1+1))
        M=(1<<(i.bit_length()))-1; lowest=(M>>1)+1; lowest2=(M>>2)+1 if M>1 else None
        if not (lowest2 and i>=lowest2+63): continue
        w=rng.integers(0,2**32,64,dtype=np.uint64)
        c=i-lowest
        vh=i-(w & M).astype(np.int64); vl=i-(w & (M>>1)).astype(np.int64)
        lanes=np.arange(64)
        def f(acc):
            rk=np.concatenate([[0],np.cumsum(acc)[:-1]])
            v=np.where(rk<=c, vh, vl)
            return rk<=v
        a0=init(i,M,vh,vl,c,lanes)
        iters=0
        while True:
            a1=f(a0); a2=f(a1); iters+=1
            if (a1==a2).all(): break
            a0=a2
        it_hist.append(iters)
    h=np.bincount(it_hist); return h/ h.sum(), np.mean(it_hist)
cur=lambda i,M,vh,vl,c,l: vh>=0
def prop(i,M,vh,vl,c,l):
    p=(i+1-32)/(M+1)
    g=np.floor(l*p).astype(np.int64)
    v=np.where(g<=c, vh, vl)
    return g<=v
print("current", run(cur))
print("proportional", run(prop))

def rounds(init, trials=20000):
    hist=[]
    for _ in range(trials):
        i=int(rng.integers(200, n1+1))
        M=(1<<(i.bit_length()))-1; lowest=(M>>1)+1; lowest2=(M>>2)+1 if M>1 else None
        if not (lowest2 and i>=lowest2+63): continue
        w=rng.integers(0,2**32,64,dtype=np.uint64)
        c=i-lowest
        vh=i-(w & M).astype(np.int64); vl=i-(w & (M>>1)).astype(np.int64)
        lanes=np.arange(64)
        def f(acc):
            rk=np.concatenate([[0],np.cumsum(acc)[:-1]])
            v=np.where(rk<=c, vh, vl)
            return rk<=v
        a=init(i,M,vh,vl,c,lanes); t=0
        while True:
            b=f(a)
            if (b==a).all(): break
            a=b; t+=1
        hist.append(t)
    h=np.bincount(hist); return (h/h.sum())[:6], np.mean(hist)
print("rounds to fixed point (t: a_t is fixed) current", rounds(cur))
print("rounds proportional", rounds(prop))
def prop2(i,M,vh,vl,c,l):
    # exact expected rank under the per-lane accept probabilities is hard; try a two-step: rank from vh>=0 count then proportional
    a=vh>=0
    return a
