"""Test-time code optimisation + evaluation on MI355X (reference CLI: optimize.py).

  python optimize.py --saved_dir srncar --tgt_instances 1 [--splits test]
         [--num_opts 200] [--lr 1e-2] [--lr_half_interval 50] [--save_img True]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def main():
    from codenerf_amd.utils import str2bool
    ap = argparse.ArgumentParser(description="CodeNeRF")
    ap.add_argument("--gpu", dest="gpu", default=0)
    ap.add_argument("--saved_dir", dest="saved_dir", default="srncar")
    ap.add_argument("--tgt_instances", dest="tgt_instances", nargs="+", default=[1])
    ap.add_argument("--splits", dest="splits", default="test")
    ap.add_argument("--num_opts", dest="num_opts", default=200)
    ap.add_argument("--lr", dest="lr", default=1e-2)
    ap.add_argument("--lr_half_interval", dest="lr_half_interval", default=50)
    ap.add_argument("--save_img", dest="save_img", default=True)
    ap.add_argument("--jsonfile", dest="jsonfile", default="srncar.json")
    ap.add_argument("--batchsize", dest="batchsize", default=2048)
    args = ap.parse_args()

    from codenerf_amd.optimizer import Optimizer
    tgt = [int(i) for i in args.tgt_instances]
    opt = Optimizer(args.saved_dir, int(args.gpu), tgt, args.splits, args.jsonfile, int(args.batchsize),
                    int(args.num_opts))
    opt.optimize_objs(tgt, float(args.lr), int(args.lr_half_interval), str2bool(args.save_img))


if __name__ == "__main__":
    main()
