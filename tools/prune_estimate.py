"""CPU estimate behind DESIGN.md section 10 item 1: on the SURVEY section 8(d) generator (synth.py), tau (the
K = 100th Hamming distance among 24K cluster-mates of a query) vs the partial-distance lower bound
d1(first b bits) + (pc2(q) - pc2(r)) of rows from other clusters; prints the surviving fraction per b."""
import torch, math
torch.manual_seed(0)
d=1024; NC=4096
C=torch.randn(NC,d)/math.sqrt(d)
def rows(lab):
    F=C[lab]+(0.6/math.sqrt(d))*torch.randn(len(lab),d)
    return F/F.norm(dim=1,keepdim=True)
nq=32
qlab=torch.randint(0,NC,(nq,))
src=rows(qlab)
Q=src+0.3/math.sqrt(d)*torch.randn(nq,d); Q=Q/Q.norm(dim=1,keepdim=True)
qb=(Q>0)
off=rows(torch.randint(0,NC,(200000,)))>0
for frac_bits in (512,576,640,704,768):
    pass
taus=[];res={fb:[] for fb in (512,576,640,704,768)}
for i in range(nq):
    mates=rows(torch.full((24000,),int(qlab[i])))>0
    dm=(mates!=qb[i]).sum(1)
    tau=dm.sort().values[99].item()+1
    taus.append(tau)
    for fb in res:
        d1=(off[:,:fb]!=qb[i][:fb]).sum(1)
        lb=(qb[i][fb:].sum()-off[:,fb:].sum(1))  # d2 >= pc2(q) - pc2(r)
        res[fb].append(((d1+lb)<tau).float().mean().item())
print('tau',sorted(taus))
for fb in res: print(fb, 'offcluster survive frac mean', sum(res[fb])/nq, 'max', max(res[fb]))
