import sys, os
sys.path.insert(0, "mandheling-dsp-training_amd"); sys.path.insert(0, "oracle")
import numpy as np, torch
import niti_amd, niti_oracle as O
from niti_amd import ops
n, ci, h, w, co, k, s, p = 4, 1, 28, 28, 20, 5, 1, 0
g = O.geom(n, ci, h, w, co, k, stride=s, pad=p)
rng = np.random.default_rng(203)
x = O.synth_x(rng, (n, ci, h, w)); dy = O.synth_dy(rng, (n, co, g.oh, g.ow))
dw_ref, bw_ref, acc_ref = O.mnn_conv_wgrad(g, x, dy)
acc_naive, _ = O.conv_wgrad_acc(g, x, dy)
print("mnn acc == naive acc:", np.array_equal(acc_ref, acc_naive), "bw", bw_ref)
xT4 = O.nchw_to_c4(np.ascontiguousarray(x.transpose(1, 0, 2, 3)))
dyT = np.ascontiguousarray(dy.transpose(1, 0, 2, 3))
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
out4 = torch.zeros(((co + 3) // 4, ci, k, k, 4), dtype=torch.int8, device="cuda")
ex = ops.NITIExecution(niti_amd.OP_GRADIENT_CONV_INT8, ops.conv_common((g.ow, g.oh), stride=1, pad=p))
ins = [ops.tensor(dev(xT4), (ci, n, h, w), 2), ops.tensor(dev(dyT), (co, n, g.oh, g.ow))]
outs = [ops.tensor(out4, (ci, co, k, k), 2)]
print("resize", ex.resize(ins, outs), "exec", ex.execute(ins, outs))
torch.cuda.synchronize()
got = O.c4_to_nchw(out4.cpu().numpy(), co).transpose(1, 0, 2, 3)
print("equal:", np.array_equal(got, dw_ref))
print("got", got[0, 0]); print("ref", dw_ref[0, 0])
# native
gg = ops.geom(n, ci, h, w, co, k, stride=s, pad=p)
acc = ops.conv_wgrad_acc(gg, ops.nchw_to_chwn16(dev(x)), ops.nchw_to_chwn16(dev(dy))).cpu().numpy()
print("native acc ok:", np.array_equal(acc[..., :ci].transpose(0, 3, 1, 2), acc_naive))
print("native acc[0,:,:,0]", acc[0, :, :, 0]); print("ref acc", acc_naive[0, 0])
