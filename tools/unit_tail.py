#!/usr/bin/env python3
"""Tail analysis of the persistent render from a VRT_UNIT_DIAG build's dumps
(gpurun_out/unit_diag_<i>.bin: per unit start / end s_memrealtime ticks,
wave, slice): launch span, time-averaged busy waves / peak ("eff"), when the
busy count last stood at 90 % / 50 % of its peak, unit durations, and when
the waves ran dry.  usage: tools/unit_tail.py 0 3 8 12
"""
import numpy as np, sys
for i in [int(x) for x in sys.argv[1:]]:
    d=np.fromfile(f'gpurun_out/unit_diag_{i}.bin',dtype=np.uint32).reshape(-1,4).astype(np.int64)
    s=d[:,0]; e=d[:,1]; ref=s[0]
    s=((s-ref+2**31)&0xffffffff)-2**31; e=((e-ref+2**31)&0xffffffff)-2**31
    b0=s.min(); s=s-b0; e=e-b0; T=e.max()
    ev=np.concatenate([np.stack([s,np.ones_like(s)],1),np.stack([e,-np.ones_like(e)],1)])
    ev=ev[np.lexsort((ev[:,1],ev[:,0]))]
    busy=np.cumsum(ev[:,1]); tt=ev[:,0]
    area=np.sum(busy[:-1]*np.diff(tt)); peak=busy.max()
    t90=tt[np.where(busy>=0.9*peak)[0].max()]; t50=tt[np.where(busy>=0.5*peak)[0].max()]
    wave=d[:,2]; wend=np.zeros(wave.max()+1); np.maximum.at(wend,wave,e); wend=wend[wend>0]
    wst=np.full(wave.max()+1, 1<<40); np.minimum.at(wst,wave,s); wst=wst[wst<(1<<40)]
    dur=e-s
    print(f"launch {i}: span {T/100:.1f} us, peak busy {peak}, eff {area/T/peak:.3f}, last>=90% {t90/T:.3f}, >=50% {t50/T:.3f}; unit us pcts {(np.percentile(dur,[50,90,99,100])/100).round(1)}; wave start us pcts {(np.percentile(wst,[50,99,100])/100).round(1)} end frac pcts {np.percentile(wend/T,[1,10,50,90]).round(3)}")
    # by xcd (slice x = d[:,3])
    x=d[:,3]
    print("   units taken per slice", np.bincount(x).tolist(), " help units (slice != block xcd):", int(np.sum(x != ((d[:,2]//4)&7))))
