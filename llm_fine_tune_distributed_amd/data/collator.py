"""Collation, distributed batch sampling and the prefetching loader (reference D4).

* ``SFTCollator``: right-padding with ``pad_token_id`` (= eos, training.py:94), labels = ids with
  pads -> -100, ``num_items`` = non-ignored *shifted* label count (HF ``num_items_in_batch``);
  or padding-free packing (varlen ``cu_seqlens``/``position_ids``, numerically identical per
  sample, no pad FLOPs). Both call the native CPU kernels of ``csrc/data_pipeline.cpp``.
* ``DistributedBatchSampler``: Accelerate ``BatchSamplerShard`` semantics — the base sampler is
  a seeded shuffle reshuffled every epoch; rank r takes batches r, r+W, r+2W, ...; drop_last
  keeps every rank's batch count equal (C11: no communication).
* ``DataLoader``: a background thread collates and pins the next batches; the H2D copy is
  non-blocking (training.py:277 ``dataloader_pin_memory=True``).
"""
from __future__ import annotations

import queue
import threading
from typing import Dict, Iterator, List, Optional

import torch

from ..ops import _ext
from .dataset import TokenizedDataset


class SFTCollator:
    def __init__(self, pad_token_id: int, pad_to_multiple_of: Optional[int] = None, max_length: Optional[int] = None,
                 packing: bool = False, max_tokens: Optional[int] = None):
        self.pad_token_id = int(pad_token_id)
        self.pad_to_multiple_of = int(pad_to_multiple_of or 1)
        self.max_length = int(max_length or 0)
        self.packing = packing
        self.max_tokens = max_tokens

    def max_batch_tokens(self, ds: TokenizedDataset, batch_size: int) -> int:
        """Hard upper bound of ``input_ids.numel()`` for any batch of ``batch_size`` samples of ``ds``, from the data
        actually held (not from ``max_length``, which a pre-tokenized dataset need not respect): padded batches are
        ``batch_size`` x the longest (truncated) sample rounded up to the pad multiple; packed ones the sum of the
        ``batch_size`` longest samples (or ``max_tokens``) rounded up the same way."""
        lens = ds.lengths().to(torch.int64)
        if lens.numel() == 0:
            return 0
        m = self.pad_to_multiple_of
        rup = lambda x: -(-max(int(x), 1) // m) * m  # noqa: E731
        if self.packing:
            if self.max_tokens:
                return rup(self.max_tokens)
            k = min(int(batch_size), lens.numel())
            return rup(int(torch.topk(lens, k).values.sum()))
        L = int(lens.max())
        if self.max_length:
            L = min(L, self.max_length)
        return int(batch_size) * rup(L)

    def __call__(self, ds: TokenizedDataset, indices: torch.Tensor) -> Dict:
        indices = indices.to(torch.int64)
        if self.packing:
            return self._pack(ds, indices)
        return self._pad(ds, indices)

    def _pad(self, ds, idx):
        if _ext.load():
            ids, labels, lengths = _ext.ops().pad_batch(ds.tokens, ds.offsets, idx, self.pad_token_id,
                                                        self.pad_to_multiple_of, self.max_length)
        else:
            ids, labels, lengths = _pad_py(ds, idx, self.pad_token_id, self.pad_to_multiple_of, self.max_length)
        if ds.loss_start is not None:
            st = ds.loss_start[idx].to(torch.int64)
            pos = torch.arange(ids.shape[1])[None, :]
            labels = labels.masked_fill(pos < st[:, None], -100)
        num_items = int((labels[:, 1:] != -100).sum())
        return {"input_ids": ids, "labels": labels, "num_items": num_items, "num_samples": int(idx.numel()),
                "num_tokens": int(lengths.sum())}

    def _pack(self, ds, idx):
        mt = self.max_tokens or int(ds.lengths()[idx].sum())
        if _ext.load():
            ids, labels, cu, pos, used = _ext.ops().pack_sequences(ds.tokens, ds.offsets, idx, mt, self.pad_token_id,
                                                                   self.pad_to_multiple_of)
        else:
            ids, labels, cu, pos, used = _pack_py(ds, idx, mt, self.pad_token_id, self.pad_to_multiple_of)
        n = int(used[0])
        if ds.loss_start is not None:
            seq_start = cu[:-1].to(torch.int64)
            for s in range(n):  # mask prompt tokens (labels are already shifted: position t predicts t+1)
                a = int(seq_start[s])
                ls = int(ds.loss_start[idx[s]])
                labels[a:a + max(0, ls - 1)] = -100
        lens = (cu[1:] - cu[:-1])
        return {"input_ids": ids, "labels": labels, "cu_seqlens": cu, "position_ids": pos,
                "max_seqlen": int(lens.max()), "num_items": int((labels != -100).sum()), "num_samples": n,
                "num_tokens": int(cu[n]) if n < cu.numel() else int(cu[-1]), "shifted": True}


def _pad_py(ds, idx, pad_id, mult, max_length):
    seqs = [ds[int(i)] for i in idx]
    if max_length:
        seqs = [s[:max_length] for s in seqs]
    T = max(1, max(len(s) for s in seqs))
    T = (T + mult - 1) // mult * mult
    ids = torch.full((len(seqs), T), pad_id, dtype=torch.int64)
    labels = torch.full((len(seqs), T), -100, dtype=torch.int64)
    for b, s in enumerate(seqs):
        ids[b, :len(s)] = torch.tensor(s)
        labels[b, :len(s)] = torch.tensor(s)
    return ids, labels, torch.tensor([len(s) for s in seqs], dtype=torch.int32)


def _pack_py(ds, idx, max_tokens, pad_id, mult):
    ids, labels, pos, cu = [], [], [], [0]
    used = 0
    for i in idx.tolist():
        s = ds[i][:max_tokens] if max_tokens else ds[i]
        if max_tokens and cu[-1] + len(s) > max_tokens and used > 0:
            break
        ids += s
        labels += s[1:] + [-100]
        pos += list(range(len(s)))
        cu.append(cu[-1] + len(s))
        used += 1
    M = cu[-1]
    Mp = (max(M, 1) + mult - 1) // mult * mult
    if Mp > M:
        ids += [pad_id] * (Mp - M)
        labels += [-100] * (Mp - M)
        pos += list(range(Mp - M))
        cu.append(Mp)
    return (torch.tensor(ids, dtype=torch.int64), torch.tensor(labels, dtype=torch.int64),
            torch.tensor(cu, dtype=torch.int32), torch.tensor(pos, dtype=torch.int64), torch.tensor([used]))


class DistributedBatchSampler:
    def __init__(self, n: int, batch_size: int, world_size: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 42, drop_last: bool = True):
        self.n, self.bs, self.ws, self.rank = n, batch_size, world_size, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0

    def set_epoch(self, e: int):
        self.epoch = e

    def _batches(self) -> List[torch.Tensor]:
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        bs = list(order.split(self.bs))
        if self.drop_last and bs and bs[-1].numel() < self.bs:
            bs = bs[:-1]
        return bs

    def __len__(self):
        nb = len(self._batches())
        return nb // self.ws if self.drop_last else (nb + self.ws - 1) // self.ws

    def __iter__(self) -> Iterator[torch.Tensor]:
        bs = self._batches()
        per = len(self)
        for i in range(per):
            j = i * self.ws + self.rank
            if j < len(bs):
                yield bs[j]
            else:  # uneven tail without drop_last: wrap around like Accelerate's even_batches
                yield bs[j % len(bs)]


class DataLoader:
    """Iterates device-ready micro-batches; collation + pinning run in a background thread."""

    def __init__(self, ds: TokenizedDataset, collator: SFTCollator, sampler: DistributedBatchSampler,
                 device: torch.device, pin_memory: bool = True, prefetch: int = 2):
        self.ds, self.collator, self.sampler = ds, collator, sampler
        self.device = device
        self.pin = pin_memory and device.type == "cuda"
        self.prefetch = max(1, prefetch)

    def __len__(self):
        return len(self.sampler)

    def set_epoch(self, e):
        self.sampler.set_epoch(e)

    def _host_batches(self, skip: int = 0):
        for k, idx in enumerate(self.sampler):
            if k < skip:
                continue
            b = self.collator(self.ds, idx)
            # the token count travels with the batch (pinned, non-blocking H2D): building it on the device
            # later from a Python number is a pageable copy that stalls the host at every step
            b["num_items_t"] = torch.tensor([float(b["num_items"])], dtype=torch.float32)
            if self.pin:
                b = {k2: (v.pin_memory() if torch.is_tensor(v) else v) for k2, v in b.items()}
            yield b

    def iter(self, skip: int = 0):
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        sentinel = object()
        stop = threading.Event()

        def put(item) -> bool:  # False once the consumer has gone away
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    continue
            return False

        def work():
            try:
                for b in self._host_batches(skip):
                    if not put(b):
                        return
            except BaseException as e:  # surface errors in the main thread
                put(e)
            put(sentinel)

        t = threading.Thread(target=work, name="sftamd-collate", daemon=True)
        t.start()
        try:
            while True:
                b = q.get()
                if b is sentinel:
                    break
                if isinstance(b, BaseException):
                    raise b
                yield {k: (v.to(self.device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in b.items()}
        finally:
            # a consumer that stops early (max_steps inside an epoch, an exception) closes the generator: the
            # producer must not stay parked on a full queue holding its pinned batches for the life of the process
            stop.set()
            t.join()

    def __iter__(self):
        return self.iter(0)
