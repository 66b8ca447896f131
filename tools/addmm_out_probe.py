import torch
a=torch.randn(64,32,device="cuda").bfloat16(); b=torch.randn(32,16,device="cuda").bfloat16(); c=torch.randn(64,16,device="cuda")
o=torch.empty(64,16,device="cuda")
r=torch.addmm(c,a,b,out_dtype=torch.float32,out=o)
print("out= ok", r.data_ptr()==o.data_ptr(), float((o-(c+(a.float()@b.float()))).abs().max()))
