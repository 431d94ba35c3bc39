import sys, torch, json
sys.path[:0]=['/root/repo','/root/repo/dfc-sa-unet_amd']
import torch.nn.functional as F
import dfcsa
from dfcsa import ops
def rel(a,b): a,b=a.double().cpu(),b.double().cpu(); return ((a-b).norm()/b.norm()).item()
def nhwc(x,dt): return x.permute(0,2,3,1).contiguous().to('cuda',dt)
out=[]
for dtype in (torch.float32, torch.bfloat16):
  for (B,Cs,nsrc,C,H) in [(3,64,2,64,14),(2,32,1,136,20)]:
    for knobs in [(0,0,1),(1,4,1),(1,8,1),(0,4,1),(0,8,0)]:
      for fuse in (0,-1):
        torch.manual_seed(3)
        xs=[torch.randn(B,Cs,H,H).to(dtype).float() for _ in range(nsrc)]
        x=torch.cat(xs,1); w=torch.randn(C,nsrc*Cs,3,3,requires_grad=True); g=torch.randn(B,C,H,H).to(dtype).float()
        F.conv2d(x,w,padding=1).backward(g)
        xh=[nhwc(t,dtype) for t in xs]; segs=[(t,kh-1,kw-1) for kh in range(3) for kw in range(3) for t in xh]
        gw=torch.zeros(C,nsrc*Cs,3,3,device='cuda')
        dfcsa.set_tuning(7,knobs[0]); dfcsa.set_tuning(6,knobs[1]); dfcsa.set_tuning(8,knobs[2]); dfcsa.set_tuning(12,fuse)
        ops.conv_wgrad_into(dtype,[nhwc(g,dtype)],C,segs,Cs,(B,H,H),(H,H),[gw],9,nsrc*Cs,nsrc*Cs); torch.cuda.synchronize()
        dfcsa.set_tuning(7,0); dfcsa.set_tuning(6,0); dfcsa.set_tuning(8,1); dfcsa.set_tuning(12,0)
        print(json.dumps({"dt":str(dtype),"shape":[B,Cs,nsrc,C,H],"knobs":knobs,"fuse":fuse,"rel":rel(gw,w.grad)}),flush=True)
