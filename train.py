"""CodeNeRF training on MI355X (reference CLI: train.py).

  python train.py --jsonfile srncar.json --save_dir srncar [--gpu 0]
         [--iters_crop N] [--iters_all N] [--batchsize 2048] [--num_instances_per_obj 2]
  python train.py --synthetic 8        # write a synthetic SRN-format split first

Multi-GPU (one process per GPU, gradients all-reduced over RCCL):
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser(description="CodeNeRF")
    ap.add_argument("--gpu", dest="gpu", default=int(os.environ.get("LOCAL_RANK", 0)))
    ap.add_argument("--save_dir", dest="save_dir", default="srncar")
    ap.add_argument("--iters_crop", dest="iters_crop", default=1000000)
    ap.add_argument("--iters_all", dest="iters_all", default=1200000)
    ap.add_argument("--batchsize", dest="batchsize", default=2048)
    ap.add_argument("--jsonfile", dest="jsonfile", default="srncar.json")
    ap.add_argument("--num_instances_per_obj", dest="num_instances_per_obj", default=2)
    ap.add_argument("--synthetic", type=int, default=0,
                    help="first write a synthetic SRN-format split with this many objects to the JSON's data_dir")
    args = ap.parse_args()

    from codenerf_amd.trainer import Trainer, load_hpams
    hp = load_hpams(args.jsonfile)
    if args.synthetic:
        from codenerf_amd.data import make_synthetic_srn
        d = hp["data"]
        make_synthetic_srn(d["data_dir"], d["cat"], d["splits"], n_obj=args.synthetic,
                           radius=2.0 if "chair" in d["cat"] else 1.3)
    dist = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(int(args.gpu))
        dist.init_process_group("nccl", device_id=torch.device("cuda", int(args.gpu)))
    trainer = Trainer(args.save_dir, int(args.gpu), hpams=hp, batch_size=int(args.batchsize), dist=dist)
    trainer.training(int(args.iters_crop), int(args.iters_all), int(args.num_instances_per_obj))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
