import torch, time
x = torch.empty(6*2**30//2, dtype=torch.float16, device='cuda')
for _ in range(3): x.fill_(1.0)
torch.cuda.synchronize(); t=time.time()
for _ in range(10): x.fill_(0.5)
torch.cuda.synchronize(); dt=(time.time()-t)/10
print("fill 6 GiB: %.3f ms  %.2f TB/s" % (dt*1e3, x.numel()*2/dt/1e12))
