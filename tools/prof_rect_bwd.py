import sys, torch
sys.path.insert(0, ".")
import __graft_entry__ as ge
pkg = ge.load_package()
dev = torch.device("cuda:0")
big = 16 * 1024 * 1024
torch.manual_seed(0)
_, _, bs, bt, sc, dv = pkg.adjust(dev, big)
g = torch.randn(big, 3, 3, device=dev)
for T in (16, 1):
    for _ in range(10):
        pkg.tensor_aca_rect_backward(bs, bt, g, sc, dv, True, True, aten_threads=T)
torch.cuda.synchronize()
print("ok")
