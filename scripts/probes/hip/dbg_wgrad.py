import torch
from distributed_resnet_tensorflow_amd.ops.backend import HipBackend, RefBackend, ConvGeom
hip, ref = HipBackend(), RefBackend()
torch.set_printoptions(linewidth=200, precision=2)
def run(N,H,C,K,R,s,p, mode):
    P = H if s==1 else (H-1)//s+1
    if mode=='ones':
        x = torch.zeros(N,H,H,C); x[...,0]=1
        dy = torch.zeros(N,P,P,K); dy[...,0]=1
    elif mode=='pix':
        x = torch.zeros(N,H,H,C); x[0,0,0,:]=torch.arange(C).float()
        dy = torch.zeros(N,P,P,K); dy[0,0,0,:]=1+torch.arange(K).float()
    else:
        x = torch.randn(N,H,H,C).bfloat16().float(); dy=torch.randn(N,P,P,K).bfloat16().float()
    dw_ref = torch.zeros(K,R,R,C); ref.conv_wgrad(x, dy, dw_ref, ConvGeom(s,p,p))
    dw = torch.zeros(K,R,R,C, device='cuda')
    ws = torch.zeros(max(1,hip.wgrad_ws_elems(N*P*P,K,R,R,C)), device='cuda')
    hip.conv_wgrad(x.bfloat16().cuda(), dy.bfloat16().cuda(), dw, ConvGeom(s,p,p), ws=ws)
    torch.cuda.synchronize()
    dw = dw.cpu()
    print(mode, (N,H,C,K,R), 'err', ((dw-dw_ref).norm()/dw_ref.norm()).item())
    if mode != 'rand':
        print('ref\n', dw_ref.reshape(K,-1)[:16,:16]); print('hip\n', dw.reshape(K,-1)[:16,:16])
run(1,4,8,16,1,1,0,'ones')
run(1,4,8,16,1,1,0,'pix')
run(1,4,8,16,1,1,0,'rand')
run(2,8,64,64,1,1,0,'rand')
