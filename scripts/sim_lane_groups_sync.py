"""Lane-group cursor model with exact resynchronisation (CPU simulation, diagnostic;
round 3): each 8x8 block decoded by L lanes of one wave, lane k
starting at bit off + k*len/L (lane 0 exact, the others speculative). Lane k >= 1 is
in sync from the first of its symbol boundaries that lies on the block's true path
(Huffman paths re-synchronise); its earlier symbols are garbage it still has to step
through. Each lane decodes from its start to the next synced lane's sync point (the
last lane to the block end); a lane that never syncs inside the block hands its
segment to the lane before it. The numbers are serial decode steps per lane; a wave
(64/L blocks) runs as long as its slowest lane, and a single-frame launch (all waves
at once, one or a few per SIMD) as long as its slowest wave.

    python scripts/sim_lane_groups_sync.py

BigBridge (round 3): L=1 64 steps everywhere; L=2 block mean 37.4, wave max p50 55 /
p90 64 / p99 64 / max 64; L=3 p50 44 / p90 54 / max 64; L=4 p50 39 / p90 50 / p99 61 /
max 65 (3,383 blocks never resync). The frame's slowest wave keeps 64 steps.
"""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import metalhuffman_amd as mh
from metalhuffman_amd import frames as F
from oracle import oracle as O
bb=F.bigbridge()
ef=mh.encode_frame(bb)
single=O.single_table(ef.canon).reshape(65536,2)
W=single[:,1].astype(np.int64)
bits=np.unpackbits(ef.codes)
n=bits.size-16
wv=np.zeros(n,np.int64)
for k in range(16): wv=(wv<<1)|bits[k:k+n]
width=W[wv]; width[width==0]=1
offs=ef.block_offsets.astype(np.int64); nb=offs.size
ends=np.append(offs[1:], offs[-1]+64*16)
p=offs[-1]
for _ in range(64): p+=width[p]
ends[-1]=p
lens=ends-offs
print("bits/block mean",lens.mean(),"max",lens.max())
def walk(start, stop_at, maxsteps=300):
    P=start.copy(); cnt=np.zeros_like(P); 
    paths=[]
    for _ in range(maxsteps):
        live=P<stop_at
        if not live.any(): break
        paths.append(np.where(live,P,-1))
        P=np.where(live,P+width[np.minimum(P,width.size-1)],P); cnt+=live
    return cnt, np.stack(paths,1) if paths else None
# true boundaries per block
for L in (2,3,4):
    starts=[offs+(lens*k)//L for k in range(L)]
    # true path positions
    cnt_true, tp = walk(offs, ends)
    assert (cnt_true==64).all()
    # per lane k>=1: its path from starts[k] to ends; sync point = first of its boundaries that is a true boundary
    steps=np.zeros((nb,L),np.int64)
    fail=np.zeros(nb,bool)
    truesets=[set(tp[i][tp[i]>=0].tolist()) for i in range(nb)]
    syncs=[None]*L
    for k in range(1,L):
        _, pk = walk(starts[k], ends)
        sk=np.zeros(nb,np.int64); garbage=np.zeros(nb,np.int64)
        for i in range(nb):
            row=pk[i][pk[i]>=0]
            hit=next((g for g,p in enumerate(row) if p in truesets[i]), None)
            if hit is None: fail[i]=True; sk[i]=ends[i]; garbage[i]=len(row)
            else: sk[i]=row[hit]; garbage[i]=hit
        syncs[k]=(sk,garbage)
    # lane k decodes from starts[k] until it reaches sync_{k+1} (for k<L-1) or the end (k=L-1)
    # lane k's steps = garbage_k + true symbols from sync_k to sync_{k+1}
    tpos=[np.array(sorted(s)) for s in truesets]
    def ntrue(i,a,b): # true symbols with start in [a,b)
        t=tpos[i]; return np.searchsorted(t,b)-np.searchsorted(t,a)
    for i in range(nb):
        sy=[offs[i]]+[syncs[k][0][i] for k in range(1,L)]+[ends[i]]
        g=[0]+[syncs[k][1][i] for k in range(1,L)]
        # if lane k failed to sync, lane k-1 covers its segment (chain): model by merging
        ok=[True]+[syncs[k][0][i]<ends[i] for k in range(1,L)]
        lane_steps=[0]*L
        for k in range(L):
            if not ok[k]:
                lane_steps[k]=g[k]; continue
            # next lane that synced
            j=k+1
            while j<L and not ok[j]: j+=1
            nxt=sy[j] if j<L else ends[i]
            lane_steps[k]=g[k]+ntrue(i,sy[k],nxt)
        steps[i,:]=lane_steps
    bm=steps.max(1)
    bpw=64//L
    nw=-(-nb//bpw); sp=np.zeros(nw*bpw,np.int64); sp[:nb]=bm
    wm=sp.reshape(nw,bpw).max(1)
    print(f"L={L}: sync fails {fail.sum()}, block max-lane steps mean {bm.mean():.1f} p99 {np.percentile(bm,99):.0f} max {bm.max()}; wave max p50 {np.median(wm):.0f} p90 {np.percentile(wm,90):.0f} p99 {np.percentile(wm,99):.0f} max {wm.max()}")
