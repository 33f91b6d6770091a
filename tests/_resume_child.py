"""Child process of ``test_engine_gpu.py::test_resume_in_new_process_replays_kernel_choices``:
pre-seeds this fresh process's kernel-choice tables with choices OTHER than the writer's (so a
checkpoint that did not carry its table would run other kernels), restores the checkpoint, runs two
steps and saves the master vector. argv: checkpoint, writer's table (JSON), output file."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from garfield_amd import _native  # noqa: E402
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.ops import grouped as gm  # noqa: E402
from garfield_amd.ops import tuning  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402
from garfield_amd.utils.checkpoint import load_engine  # noqa: E402


def main():
    ck, table_path, out = sys.argv[1:4]
    with open(table_path) as fh:
        table = json.load(fh)
    C_ = _native.native()
    for k, v in table["gemm"]:
        M, N, K, rg, add, pro = k
        alt = [c for c in range(C_.gemm_nt_num_cfg()) if c != v and C_.gemm_nt_valid(c, N, K)
               and (rg == 0 or C_.gemm_nt_stats_rows(c) <= rg) and not pro]
        gm._GEMM_CFG[tuning._tup(k)] = alt[0] if alt else v
    for k, v in table["s2"]:
        gm._S2_CHOICE[tuning._tup(k)] = False            # the dcol GEMM + col2im always applies
    for k, v in table["scwg"]:
        gm._SC_WG_CHOICE[tuning._tup(k)] = not v if v else True   # (the dense form always applies)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("resnet50"), F.cross_entropy, DistContext(device=dev),
                             EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.02, cuda_graph=True))
    load_engine(ck, eng)
    batches = synthetic_batches(5, 8, (3, 32, 32), 10, dev)
    for _ in range(2):
        eng.step(batches)
    torch.cuda.synchronize()
    torch.save({"flat": eng.flat_model().cpu(), "table": tuning.export()}, out)


if __name__ == "__main__":
    main()
