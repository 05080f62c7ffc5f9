import ctypes, sys, os, torch
sys.path.insert(0, '/root/repo' if os.path.isdir('/root/repo') else os.getcwd())
import crosscoder_amd
from crosscoder_amd import _lib
L=_lib.load_debug()  # (the pp_mask setter lives in the test-only debug build)
dev=torch.device('cuda:0'); g=torch.Generator(device=dev).manual_seed(0)
B,h=4096,16384
st=ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P=lambda t: ctypes.c_void_p(t.data_ptr())
acts=torch.relu(torch.randn(B,h,device=dev,generator=g)).to(torch.bfloat16)
res={}
for Kn in (4608, 4096, 512):
    W=(torch.randn(h,Kn,device=dev,generator=g)*0.02).to(torch.bfloat16)
    rec=torch.empty(B,Kn,device=dev)
    for mask in (5,7):
        L.cc_debug_set_pp_mask(mask)
        fn=lambda: L.cc_decode_fwd(P(acts),P(W),None,P(rec),None,B,h,Kn,1,st)
        for _ in range(3): assert fn()==0
        ts=[]
        for r in range(5):
            s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10): fn()
            e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e)/10)
        ts.sort(); med=ts[2]
        print(f"G2 N={Kn} mask={mask}: {med*1e3:.1f} us  {2*B*h*Kn/med/1e9:.0f} TF/s")
