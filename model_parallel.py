"""Model parallelism (reference 03.model_parallel.ipynb).

  python model_parallel.py toy                 # ToyModel split over 2 devices, one SGD step
  python model_parallel.py resnet [--repeat 10] # MP vs pipelined vs single-GPU ResNet-50 benchmark + bar chart
  python model_parallel.py placement           # device_map-style Llama placement (+ int8) report
  torchrun --nproc-per-node 2 model_parallel.py sendrecv   # 2-rank stage split over RCCL send/recv

With one visible GPU both stages run on cuda:0 (the split logic is unchanged); ``--cpu`` forces CPU.
"""
import argparse
import json

import torch


def _devs(args):
    if args.cpu or not torch.cuda.is_available():
        return ("cpu", "cpu")
    n = torch.cuda.device_count()
    return ("cuda:0", "cuda:1" if n > 1 else "cuda:0")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("what", choices=["toy", "resnet", "placement", "sendrecv"])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--repeat", type=int, default=10)
    ap.add_argument("--split_sizes", default="20", help="pipeline micro-batch sizes, comma list")
    ap.add_argument("--channels_last", action="store_true")
    ap.add_argument("--cudnn_benchmark", default="auto", choices=["auto", "on", "off"],
                    help="resnet: MIOpen exhaustive solver find in the warm-up train() (auto: with --channels_last; "
                         "the NCHW fp32 search runs minutes)")
    ap.add_argument("--fig", default="mp_vs_single.png")
    ap.add_argument("--json", default=None)
    ap.add_argument("--devices", type=int, default=4, help="placement: number of devices to plan for")
    ap.add_argument("--micro_batches", type=int, default=4)
    a = ap.parse_args(argv)
    from pytorch_distributed_training_tutorials_amd.apps import model_parallel as mp

    if a.what == "toy":
        d0, d1 = _devs(a)
        print(f"loss {mp.toy_step(d0, d1):.6f}")
    elif a.what == "resnet":
        import torch

        torch.backends.cudnn.benchmark = a.cudnn_benchmark == "on" or (a.cudnn_benchmark == "auto" and a.channels_last)
        res = mp.benchmark(a.repeat, _devs(a), tuple(int(s) for s in a.split_sizes.split(",") if s),
                           a.channels_last, a.fig, a.json)
        print(json.dumps(res, indent=1))
    elif a.what == "placement":
        from pytorch_distributed_training_tutorials_amd.models.llama import build_llama
        from pytorch_distributed_training_tutorials_amd.parallel.placement import infer_device_map

        # plan on the meta device (nothing allocated); int8 projections weigh 1 byte per weight
        m = build_llama("7b", dtype=torch.float16, device="meta")
        dmap = infer_device_map(m, [f"cuda:{i}" for i in range(a.devices)], linear_weight_bytes=1)
        for name, dev in dmap.items():
            print(f"{name:40s} -> {dev}")
    elif a.what == "sendrecv":
        import torch.nn as nn

        from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
        from pytorch_distributed_training_tutorials_amd.parallel import env
        from pytorch_distributed_training_tutorials_amd.parallel.pipeline import PipelineStage

        env.init_process_group("nccl")
        dev = env.device()
        rank = env.rank()
        torch.manual_seed(0)
        net1, net2 = nn.Linear(10000, 10), nn.Linear(10, 5)
        stage = (nn.Sequential(net1, nn.ReLU()) if rank == 0 else net2).to(dev)
        st = PipelineStage(stage, comm_mod.get_default(dev if dev.type == "cuda" else None),
                           loss_fn=nn.MSELoss(), micro_batches=a.micro_batches)
        opt = torch.optim.SGD(stage.parameters(), lr=1e-3)
        for it in range(3):
            x = torch.randn(20, 10000)
            y = torch.randn(20, 5)
            opt.zero_grad()
            loss = st.train_step(x if rank == 0 else None, y if rank == env.world_size() - 1 else None)
            opt.step()
            if loss is not None:
                print(f"[rank {rank}] step {it} loss {float(loss):.6f}")
        env.destroy_process_group()


if __name__ == "__main__":
    main()
