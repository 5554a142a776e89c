import numpy as np
def ref(p, luma):
    if luma: v=(p*2441856-38008785)>>21
    else: v=(p*596864-9027848)>>19
    return min(max(v,0),255)
def f32(x): return float(np.float32(x))
kM=12582912.0
for luma in (True, False):
    A,B,S = (2441856,38008785,21) if luma else (596864,9027848,19)
    a=f32(A/2**S); assert a==A/2**S
    best=None
    # search c near -(B/2^S) - 0.5 over nearby fp32 values
    c0=f32(-B/2**S-0.5)
    cands=[c0]
    x=np.float32(c0)
    for k in range(1,64):
        cands.append(float(np.nextafter(np.float32(cands[-1]),np.float32(0))))
    y=np.float32(c0)
    for k in range(1,64):
        y=np.nextafter(y,np.float32(-100)); cands.append(float(y))
    ok=[]
    for c in cands:
        good=True
        for p in range(256):
            r=f32(p*a+c)          # fma: exact product+sum in float64, one rounding
            v=f32(r+kM)           # RNE at ulp 1
            v=min(max(v,kM),kM+255)
            if int(v-kM)!=ref(p,luma): good=False;break
        if good: ok.append(c)
    print('luma' if luma else 'chroma', 'a', a, 'c0', c0, 'ok', len(ok), ok[:3], (min(ok),max(ok)) if ok else None)
