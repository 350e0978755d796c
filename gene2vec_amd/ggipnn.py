"""GGIPNN AUC harness -- PyTorch restatement of the reference's TF1 classifier.

Consumer of the exporter's .txt matrix; TensorFlow 1
is absent here, so the model is restated in PyTorch with the same data
pipeline, architecture, initialisers and optimiser:

  data   src/GGIPNN_Classification.py:43-96 -- splitlines() of the six files,
         vocabulary over train+valid+test (GGIPNN_util.myFitDict, first
         occurrence over lines with exactly 2 space-separated genes), ids via
         myFit (lines without 2 genes stay [1, 1]), one-hot labels
  embed  GGIPNN_util.load_embedding_vectors: U(-0.25, 0.25) then rows found in
         the .txt (line.split()); frozen (train_embedding=False, GGIPNN.py:19-21)
  model  GGIPNN.py:25-69 -- concat(2 x D) -> 100 -> 100 -> 10 -> 2, ReLU,
         dropout keep 0.5 after each hidden layer, biases 0.1, weights
         variance_scaling (factor 2, fan_in, truncated normal)
  train  Adam(1e-3), batch 128, 1 epoch, softmax cross-entropy, l2 = 0
         (GGIPNN_Classification.py:15-30,123-127,208-221)
  score  test AUC of softmax[:, 1] (sklearn roc_auc_score, :238-254)

Randomness (unseeded in the reference) is driven by one ``seed`` here.
"""
from __future__ import annotations

import math
import os

import numpy as np


def read_lines(path):
    with open(path, "r") as f:
        return f.read().splitlines()


def load_prediction_data(data_dir):
    sp = {}
    for part in ("train", "valid", "test"):
        sp[part] = (read_lines(os.path.join(data_dir, f"{part}_text.txt")),
                    read_lines(os.path.join(data_dir, f"{part}_label.txt")))
    return sp


def my_fit_dict(lines, length=2):
    d = {}
    for line in lines:
        eles = line.strip().split(" ")
        if len(eles) == length:
            for e in eles:
                if e not in d:
                    d[e] = len(d)
    return d


def my_fit(lines, length, d):
    x = np.ones((len(lines), length), dtype=np.int64)
    for i, line in enumerate(lines):
        eles = line.strip().split(" ")
        if len(eles) == length:
            j = 0
            for e in eles:
                x[i, j] = d[e]
                j = 1  # (sic) GGIPNN_util.py:77 -- correct for length 2
    return x


def one_hot(labels):
    names = ["0", "1"]
    y = np.zeros((len(labels), 2), dtype=np.int64)
    for i, lab in enumerate(labels):
        y[i, names.index(lab)] = 1
    return y


def load_embedding_vectors(vocabulary, filename, vector_size, rng):
    emb = rng.uniform(-0.25, 0.25, (len(vocabulary), vector_size))
    with open(filename) as f:
        for line in f:
            values = line.split()
            word = values[0]
            if word in vocabulary:
                emb[vocabulary[word]] = np.asarray(values[1:], dtype="float32")
    return emb


def _variance_scaling_(w, gen):
    """tf.contrib.layers.variance_scaling_initializer(): factor 2, FAN_IN,
    truncated normal with stddev sqrt(1.3 * 2 / fan_in), cut at 2 stddev."""
    import torch
    fan_in = w.shape[0]
    std = math.sqrt(1.3 * 2.0 / fan_in)
    with torch.no_grad():
        t = torch.empty_like(w)
        t.normal_(0.0, 1.0, generator=gen)
        bad = t.abs() > 2.0
        while bad.any():
            t[bad] = torch.empty(int(bad.sum()), device=w.device).normal_(0.0, 1.0, generator=gen)
            bad = t.abs() > 2.0
        w.copy_(t * std)


def build_model(vocab_size, emb, embedding_size, device, gen):
    import torch
    import torch.nn as nn

    class GGIPNN(nn.Module):
        def __init__(self):
            super().__init__()
            self.W = nn.Parameter(torch.as_tensor(emb, dtype=torch.float32, device=device),
                                  requires_grad=False)
            dims = [2 * embedding_size, 100, 100, 10, 2]
            self.ws = nn.ParameterList()
            self.bs = nn.ParameterList()
            for a, b in zip(dims[:-1], dims[1:]):
                w = nn.Parameter(torch.empty(a, b, device=device))
                _variance_scaling_(w, gen)
                self.ws.append(w)
                self.bs.append(nn.Parameter(torch.full((b,), 0.1, device=device)))

        def forward(self, x, keep_prob):
            h = self.W[x].reshape(x.shape[0], -1)
            for i in range(3):
                h = torch.relu(h @ self.ws[i] + self.bs[i])
                if keep_prob < 1.0:
                    mask = (torch.rand(h.shape, device=h.device, generator=gen) < keep_prob)
                    h = h * mask / keep_prob
            return h @ self.ws[3] + self.bs[3]

    return GGIPNN()


def train_and_auc(embedding_file, data_dir, seed=0, device="cpu", embedding_size=200,
                  batch_size=128, num_epochs=1, keep_prob=0.5, lr=1e-3):
    import torch
    from sklearn import metrics

    sp = load_prediction_data(data_dir)
    xtr, ytr = sp["train"]
    xva, yva = sp["valid"]
    xte, yte = sp["test"]
    allx = xtr + xva + xte
    voca = my_fit_dict(allx, 2)
    ids = my_fit(allx, 2, voca)
    ntr, nva = len(xtr), len(xva)
    rng = np.random.RandomState(seed)
    perm = rng.permutation(ntr)  # random.shuffle(random_indices) stand-in (seeded)
    x_train = ids[:ntr][perm]
    y1h = one_hot(ytr + yva + yte)
    y_train = y1h[:ntr][perm]
    x_test = ids[ntr + nva:]
    y_test = np.argmax(y1h[ntr + nva:], axis=1)
    emb = load_embedding_vectors(voca, embedding_file, embedding_size, rng)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    model = build_model(len(voca), emb, embedding_size, device, gen)
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=lr,
                           betas=(0.9, 0.999), eps=1e-8)
    xt = torch.as_tensor(x_train, device=device)
    yt = torch.as_tensor(np.argmax(y_train, axis=1), device=device)
    n = len(xt)
    for _ in range(num_epochs):
        order = torch.as_tensor(rng.permutation(n), device=device)  # batch_iter's shuffle
        for b0 in range(0, n, batch_size):
            idx = order[b0:b0 + batch_size]
            logits = model(xt[idx], keep_prob)
            loss = torch.nn.functional.cross_entropy(logits, yt[idx])
            opt.zero_grad()
            loss.backward()
            opt.step()
    with torch.no_grad():
        scores = torch.softmax(model(torch.as_tensor(x_test, device=device), 1.0), dim=1)[:, 1]
    return float(metrics.roc_auc_score(y_test, scores.cpu().numpy()))
