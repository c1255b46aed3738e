"""Planner kernel time per operation mix (65536 robots, N=16): which phase costs."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))


def main():
    import torch
    import mpcq
    from mpcq import synth
    dev = torch.device("cuda", 0)
    B, N = 65536, 16
    rng = np.random.default_rng(0)
    gaits = np.stack([synth.gait_table(("trot", "bound", "pace")[b % 3], N) for b in range(B)])
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    st = np.zeros((B, 12)); st[:, 2] = 0.2; st[:, 6:] = rng.normal(0, .2, (B, 6))
    d = dict(state=T(st), l_feet=T(np.tile(np.vstack([np.ones((2, 4)) * .15, np.zeros((1, 4))]), (B, 1, 1))),
             v_ref=T(rng.normal(0, .3, (B, 6))), gait=T(gaits), xref=T(np.zeros((B, 12, N + 1))),
             fsteps=T(np.zeros((B, 20, 13))), rot=T(np.zeros(B), torch.int32), h_rot=T(np.full(B, .2)))
    eng = mpcq.Engine(N)
    s = torch.cuda.Stream()
    eng.set_stream(s.cuda_stream)
    torch.cuda.set_stream(s)
    for name, ops in (("roll", mpcq.PLAN_ROLL), ("footsteps", mpcq.PLAN_FOOTSTEPS),
                      ("refstates", mpcq.PLAN_REFSTATES), ("tick", mpcq.PLAN_TICK)):
        for rep in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(10):
                eng.plan_device(B, ops, i + 1, d["state"].data_ptr(), d["l_feet"].data_ptr(), d["v_ref"].data_ptr(),
                                d["gait"].data_ptr(), d["rot"].data_ptr(), d["h_rot"].data_ptr(), d["xref"].data_ptr(),
                                d["fsteps"].data_ptr(), asynchronous=True)
            e1.record(s)
            s.synchronize()
        print(f"{name:10s} {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us per launch of {B}")
    eng.close()


if __name__ == "__main__":
    main()
