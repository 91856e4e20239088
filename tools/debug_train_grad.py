"""Debug aid: per-stage comparison of the GPU training path with the oracle's autograd twin
(feat_net inputs/activations/gradients), on one golden case. Test infrastructure only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from golden_io import Golden  # noqa: E402
from model_io import model_from_golden  # noqa: E402
from oracle import apn_oracle as O  # noqa: E402
import test_hip_parity as T  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "G3"
dev = torch.device("cuda")
g = Golden(name)
m = model_from_golden(g, dev)
sub, target = T._train_setup(g, m, dev)
t = g.t("in_t").to(dev)
with torch.no_grad():
    xyz = m(t, render_kwargs=sub)["t_hat_pcd"]
lo = (xyz.min(0)[0] - 0.01).float(); hi = (xyz.max(0)[0] + 0.01).float()
m.xyz_min.copy_(lo); m.xyz_max.copy_(hi)
cap = {}


def hook(nm):
    def f(mod, inp, out):
        if inp[0].requires_grad:
            inp[0].retain_grad()
        out.retain_grad()
        cap[nm] = (inp[0], out)
    return f


for i, l in enumerate(m.feat_net):
    l.register_forward_hook(hook(f"fn{i}"))
out = m(t, render_kwargs=sub, calc_min_max=False)
loss = torch.nn.functional.mse_loss(out["rgb_marched"], target.to(dev))
loss.backward()
orc = T._oracle_for(g, m)
params = O.oracle_trainable(orc)
ocap = []


def fn(x, st):
    if x.requires_grad:
        x.retain_grad()
    ocap.append(x)
    for nm in ["feat_net.0", "feat_net.2.0", "feat_net.3.0", "feat_net.4"]:
        x = torch.nn.functional.leaky_relu(O._lin(x, st, nm), 0.01)
        x.retain_grad()
        ocap.append(x)
    return x


O.feat_net = fn
ro = O.oracle_forward_train(orc, g.t("in_t"), sub, xyz_min=lo.cpu(), xyz_max=hi.cpu(), knn_tree=False)
lref = torch.nn.functional.mse_loss(ro["rgb_marched"], target)
lref.backward()
print("loss", float(loss), float(lref))
gin = cap["fn0"][0]
d = (gin.detach().cpu() - ocap[0].detach()).abs()
print("input diff", float(d.max()))
print("input diff per col (top)", d.max(0)[0].topk(5))
print("input diff per row (top)", d.max(1)[0].topk(5))
for i, nm in enumerate(["fn1", "fn2", "fn4", "fn5"]):
    o = cap[nm][1]
    print(nm, "act diff", float((o.detach().cpu() - ocap[i + 1].detach()).abs().max()),
          "grad diff", float((o.grad.cpu() - ocap[i + 1].grad).abs().max()),
          "grad max", float(ocap[i + 1].grad.abs().max()))
gd = (cap["fn5"][1].grad.cpu() - ocap[4].grad).abs().max(1)[0]
print("out-grad diff rows top", gd.topk(5))
r = int(gd.argmax())
print("row", r, "sample", r // 8, "gpu grad", cap["fn5"][1].grad[r, :4].cpu(), "orc", ocap[4].grad[r, :4])
