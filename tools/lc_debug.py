import os, sys, ctypes
ROOT="/root/repo"; sys.path[:0]=[ROOT, ROOT+"/smoothquant-mixedprecision_amd"]
import numpy as np, torch
from smoothquant import ops, _lib
from smoothquant.fake_quant import W4A4Linear
dev=torch.device("cuda")
M,K,G=int(sys.argv[1]),int(sys.argv[2]),64
g=torch.Generator(device=dev).manual_seed(0)
lin=torch.nn.Linear(K,512,bias=False).to(dev,torch.float16)
x=torch.randn(M,K,generator=g,device=dev).half()
q=W4A4Linear.from_float(lin,weight_quant="per_group",act_quant="per_group",importance=x.float().abs().mean(0).cpu(),salient_prop=0.05,group_size=G)
pw=q.packed()
lib=_lib.load()
nb=lib.sqmp_act_workspace_bytes(M,K,pw.Kp)
ws=torch.zeros(nb,dtype=torch.uint8,device=dev)
a=torch.empty((max(256,(M+255)//256*256), pw.Kp+pw.S_pad),dtype=torch.float16,device=dev)[:M]
p=ops._p
st=lib.sqmp_quant_act(p(x),1,M,K,2,4,G,p(pw.amap),pw.Kp,p(pw.nonsal),p(pw.salient),pw.S,pw.S_pad,0,p(a),None,None,p(ws),nb,ops._stream(x))
torch.cuda.synchronize(); print("status",st)
k64=(K+63)//64*64; tiles=(K+255)//256
w=ws.view(torch.int32).cpu().numpy()
cmax=w[:k64].view(np.float32); rank=w[k64:2*k64]; 
ent_off=2*k64+k64*tiles; lc_off=ent_off+((max(pw.Kp,K)+63)//64*64)
lct=w[lc_off:lc_off+4096].view(np.uint32)
Kn=K-pw.S
cols=lct[:Kn]&0xFFFF; pos=lct[:Kn]>>16
nonsal=pw.nonsal.cpu().numpy()
xf=x.float().cpu().numpy()
colmax=np.abs(xf[:,nonsal]).max(0)
order=nonsal[np.argsort(colmax,kind="stable")]
print("lctab cols == sorted order:", np.array_equal(cols,order), "first", cols[:8], order[:8])
print("rank_by_col consistent:", np.array_equal(rank[order], np.arange(Kn)))
amap=pw.amap.cpu().numpy()
print("positions consistent:", np.array_equal(amap[pos], cols))
print("pad entries", lct[Kn:Kn+3], "W", pw.Kp+pw.S_pad)
