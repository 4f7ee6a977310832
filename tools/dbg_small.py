import sys; sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import torch
from test_model_gpu import run_case, SMALL, grad_errs
r = run_case(SMALL, 2, 210, 12, "fp32")
g, go = r["grads"]
errs, floor = grad_errs(g, go)
print("floor", floor)
for k, v in sorted(errs.items(), key=lambda kv: -kv[1])[:8]:
    print(k, v, go[k].abs().max().item())
k = "encoder.embed.conv.2.weight"
d = (g[k].double().cpu() - go[k]).abs()
print("argmax", divmod(d.argmax().item(), 9*256), d.max().item())
# error pattern by (cout, cin, tap)
d4 = d.view(256, 256, 9)
print("by tap", d4.amax(dim=(0,1)))
print("by cout top", d4.amax(dim=(1,2)).topk(5))
print("by cin top", d4.amax(dim=(0,2)).topk(5))
