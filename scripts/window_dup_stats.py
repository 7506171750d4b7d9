"""Window-duplication statistics of the subband sum: how often a trial's
window for a channel group equals the previous trial's (same shifts for all G channels), and
how many reads strict per-(wave, group) read patterns (all 8 equal / quads / pairs) would skip.
Host only (the reference's shift table).   python scripts/window_dup_stats.py C2 [G] [ntrials]
"""
import sys, numpy as np
sys.path[:0]=['radio-pulsar-utils_amd']
from pulsarutils._planner import dedispersion_plan, dedispersion_shifts
from pulsarutils.configs import CONFIGS
cfg=CONFIGS[sys.argv[1]]
G=int(sys.argv[2]) if len(sys.argv)>2 else 4
dms=dedispersion_plan(cfg.nchan,cfg.dmmin,cfg.dmmax,cfg.start_freq,cfg.bandwidth,cfg.tsamp)
ntr=int(sys.argv[3]) if len(sys.argv)>3 else dms.size
dms=dms[:ntr]
sh=np.array([dedispersion_shifts(cfg.nchan,d,cfg.start_freq,cfg.bandwidth,cfg.tsamp) for d in dms],dtype=np.int64)
ndm,nchan=sh.shape
ng=nchan//G
# per (trial pair d,d+1) per group: windows equal iff all shifts of group equal
eq = (sh[1:].reshape(ndm-1,ng,G)==sh[:-1].reshape(ndm-1,ng,G)).all(-1)  # (ndm-1, ng)
T=128; D=8
tot=0; dup=0
# per wave pattern stats at group granularity: runs
pat={'pairs':0,'quads':0,'all8':0,'none':0}
for t0 in range(0,ndm,T):
  for w in range(0,T,D):
    a=t0+w
    if a+D>ndm: continue
    for g in range(ng):
      e=eq[a:a+D-1,g]  # e[k]: trial a+k+1 == a+k
      tot+=D; dup+=e.sum()
      if e.all(): pat['all8']+=1
      elif e[0::2].all() and e[1::2][[0,2]].all() if False else (e[0] and e[2] and e[4] and e[6] and e[1] and e[5]): pat['quads']+=1
      elif e[0] and e[2] and e[4] and e[6]: pat['pairs']+=1
      else: pat['none']+=1
print(cfg.name,'G',G,'ndm',ndm,'dup frac',dup/tot, {k:v/(tot/D) for k,v in pat.items()})
# reads saved with per-(wave,group) pattern choice: all8 ->1 read, quads->2, pairs->4, none->8
n=tot/D
saved=(pat['all8']*7+pat['quads']*6+pat['pairs']*4)/(n*8)
print('read fraction saved with 4 patterns per (wave,group):',saved)
# per group position in band: dup frac by group index deciles
fr=[eq[:,g].mean() for g in range(ng)]
print('dup frac by band decile (low freq chan 0 first):',[round(float(np.mean(fr[i*ng//10:(i+1)*ng//10])),3) for i in range(10)])
