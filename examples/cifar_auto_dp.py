#!/usr/bin/env python3
"""CIFAR-10-shaped automatic data parallelism — the reference example, MI355X-native.

Reference: cifar_example/sgd-torchad_nn-cifar.lua (+ train.sh).  Same flow:
parse flags, seed, build the ConvNet (conv 3->64 5x5, ReLU, maxpool 3/3,
conv 64->64 5x5, ReLU, maxpool 3/3, 64 -> 100 -> 10), load data, ONE call to
``parallelize`` (broadcast weights, shard data, install the periodic sync),
normalise per shard, train with the SGD trainer, evaluate the full test set on
every rank, write a results file.  Differences: synthetic CIFAR-shaped data
(no network on the GPU box; the reference downloaded CIFAR-10), minibatches,
and the reference's double log-softmax is not replicated (SURVEY A-17).

    python -m madnn.launch --nproc 8 examples/cifar_auto_dp.py -data -usegpu -batchSize 1 -iterations 2
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import madnn  # noqa: E402
from madnn.models import CifarConvNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser(prefix_chars="-")
    ap.add_argument("-data", action="store_true", help="full size (32000/10000) instead of 4000/2000")
    ap.add_argument("-seed", type=int, default=1)
    ap.add_argument("-learningRate", type=float, default=1e-3)
    ap.add_argument("-batchSize", type=int, default=1, help="SYNC PERIOD in backward passes (reference semantics)")
    ap.add_argument("-minibatch", type=int, default=32)
    ap.add_argument("-weightDecay", type=float, default=0.0)
    ap.add_argument("-iterations", type=int, default=1)
    ap.add_argument("-threads", type=int, default=1)
    ap.add_argument("-usegpu", action="store_true")
    ap.add_argument("-size", type=int, default=0, help="train/test samples override (quick runs; 0 = reference sizes)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    madnn.init(device="cuda" if a.usegpu else "cpu")
    madnn.seed_all(a.seed)  # same seed everywhere (reference :48)
    t_pre = time.time()
    model = CifarConvNet()
    trsize, tesize = (32000, 10000) if a.data else (4000, 2000)
    if a.size:
        trsize, tesize = a.size, max(a.size // 2, 10)
    g = torch.Generator().manual_seed(a.seed)
    centers = torch.randn(10, 3, 32, 32, generator=g)  # synthetic but learnable classes
    ytr = torch.randint(0, 10, (trsize,), generator=g)
    yte = torch.randint(0, 10, (tesize,), generator=g)
    xtr = centers[ytr] + 0.8 * torch.randn(trsize, 3, 32, 32, generator=g)
    xte = centers[yte] + 0.8 * torch.randn(tesize, 3, 32, 32, generator=g)

    data, labels, size = madnn.parallelize(xtr, ytr, model, trsize, sync_every=a.batchSize)
    # per-shard normalisation (the reference normalises each rank's shard, :182-216)
    mean, std = data.mean((0, 2, 3), keepdim=True), data.std((0, 2, 3), keepdim=True)
    data = (data - mean) / std
    xte = (xte - mean) / std
    dev = madnn.device()
    model.to(dev)
    t_pre = time.time() - t_pre
    opt = madnn.optim.FusedSGD(model.parameters(), lr=a.learningRate, weight_decay=a.weightDecay, momentum=0.9)
    trainer = madnn.Trainer(model, torch.nn.CrossEntropyLoss(), opt, learning_rate=a.learningRate,
                            max_iteration=a.iterations, batch_size=a.minibatch, device=dev)
    t_train = time.time()
    trainer.train(data, labels)
    t_train = time.time() - t_train
    model.eval()
    conf = torch.zeros(10, 10, dtype=torch.long)
    with torch.no_grad():
        for s in range(0, tesize, 500):
            pred = model(xte[s:s + 500].to(dev)).argmax(1).cpu()
            for t, p in zip(yte[s:s + 500], pred):
                conf[t, p] += 1
    acc = conf.diag().sum().item() / conf.sum().item()
    if madnn.get_rank() == 0:
        print(conf)
        print(f"accuracy {acc * 100:.2f}%")
        name = f"SgdAuto--Size:{trsize}--Batch:{a.batchSize}.txt"
        with open(name, "w") as f:
            f.write(f"Train size: {trsize}\nTest size: {tesize}\nbatchSize (sync period): {a.batchSize}\n"
                    f"Accuracy: {acc * 100:.2f}\nLearning rate: {a.learningRate}\nThreads: {a.threads}\n"
                    f"World size: {madnn.get_world_size()}\nPre-process time: {t_pre:.2f}s\n"
                    f"Training time: {t_train:.2f}s\n")
    madnn.shutdown()


if __name__ == "__main__":
    main()
