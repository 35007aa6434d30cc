import sys, torch; sys.path.insert(0,'.')
import tiflash_amd as tfa
dev=torch.device('cuda',0)
ctx=tfa.Context(0)
for nb in (3_000_000, 10_000_000):
    g=torch.Generator(device=dev); g.manual_seed(7)
    bk=torch.randperm(nb,device=dev,generator=g).to(torch.int64)*4+1
    bpay=bk*10
    npr=2_000_000
    hit=torch.rand(npr,device=dev,generator=g)<0.5
    pk=torch.where(hit, bk[torch.randint(0,nb,(npr,),device=dev,generator=g)], torch.randint(0,1<<40,(npr,),device=dev,generator=g)*4+3)
    ppay=pk*3
    for mode in ("A","B","C"):
        j=tfa.Join(ctx,tfa.INT64,expected_build_rows=nb)
        if mode=="A":
            j.build(bk); op,ob,_=j.probe_rows(pk,[pk],0); m=op[0].shape[0]
        elif mode=="B":
            j.build(bk,payload=[bpay]); op,ob,_=j.probe_rows(pk,[ppay],1); m=op[0].shape[0]
        else:
            j.build(bk,payload=[bpay]); op,ob,_=j.probe_rows(pk,[pk],1); m=op[0].shape[0]
        print(nb, mode, j.stats(), m, int(hit.sum().item()), flush=True)
        j.close()
