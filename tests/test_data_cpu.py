"""Data pipeline: split parity with HF datasets, native collator vs Python, sampler sharding."""
import torch

from llm_fine_tune_distributed_amd.data import collator as C
from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset, train_test_split, tokenize_rows
from llm_fine_tune_distributed_amd.data.prompts import format_prompt, WILDERNESS_EXPERT_SYSTEM_PROMPT
from llm_fine_tune_distributed_amd.data.synthetic import generate_qa, write_parquet
from llm_fine_tune_distributed_amd.data.tokenizer import load_tokenizer
from llm_fine_tune_distributed_amd.ops import _ext


def test_split_matches_hf_datasets():
    import datasets
    rows = [{"full-question": f"q{i}", "answer": f"a{i}"} for i in range(2845)]
    tr, te = train_test_split(rows, test_size=0.1, seed=42)
    assert (len(tr), len(te)) == (2560, 285)  # reference sizes (README.md:125)
    hf = datasets.Dataset.from_list(rows).train_test_split(test_size=0.1, seed=42)
    assert [r["full-question"] for r in tr] == hf["train"]["full-question"]
    assert [r["full-question"] for r in te] == hf["test"]["full-question"]


def test_format_prompt_schema():
    m = format_prompt({"full-question": "For X, why?", "answer": "because"})["messages"]
    assert [x["role"] for x in m] == ["system", "user", "assistant"]
    assert m[0]["content"] == WILDERNESS_EXPERT_SYSTEM_PROMPT


def test_synthetic_qa_schema(tmp_path):
    rows = generate_qa(300, seed=1)
    assert all(r["full-question"].startswith("For ") for r in rows)
    assert max(len(r["answer"]) for r in rows) <= 406
    p = tmp_path / "qa.parquet"
    write_parquet(rows, str(p))
    from llm_fine_tune_distributed_amd.data.dataset import load_qa_parquet
    back = load_qa_parquet(str(p))
    assert back[0] == {"full-question": rows[0]["full-question"], "answer": rows[0]["answer"]}


def test_tokenizer_roundtrip_and_chat():
    tk = load_tokenizer()
    msgs = format_prompt({"full-question": "For Essential Knots and Uses, how do I tie a bowline?",
                          "answer": "Form a loop."})["messages"]
    txt = tk.apply_chat_template(msgs, tokenize=False)
    assert "<|im_start|>assistant" in txt and txt.endswith("<|im_end|>\n")
    ids = tk.apply_chat_template(msgs)
    assert tk.decode(ids) == txt
    assert tk.pad_token_id == tk.eos_token_id  # reference: pad = eos


def _ds():
    return TokenizedDataset.synthetic(20, 1000, 3, 17, seed=0)


def test_native_collator_matches_python():
    assert _ext.load()
    ds = _ds()
    idx = torch.tensor([3, 1, 7, 19])
    a = _ext.ops().pad_batch(ds.tokens, ds.offsets, idx, 5, 8, 0)
    b = C._pad_py(ds, idx, 5, 8, 0)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    a = _ext.ops().pack_sequences(ds.tokens, ds.offsets, idx, 30, 5, 8)
    b = C._pack_py(ds, idx, 30, 5, 8)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_collator_num_items():
    ds = _ds()
    col = C.SFTCollator(pad_token_id=0)
    b = col(ds, torch.tensor([0, 1]))
    lens = ds.lengths()[:2]
    assert b["num_items"] == int((lens - 1).sum())  # HF: shifted labels != -100
    col = C.SFTCollator(pad_token_id=0, packing=True)
    p = col(ds, torch.tensor([0, 1]))
    assert p["num_items"] == b["num_items"]


def test_sampler_shards_like_accelerate():
    s = [C.DistributedBatchSampler(40, 4, 2, r, shuffle=True, seed=42) for r in range(2)]
    one = C.DistributedBatchSampler(40, 4, 1, 0, shuffle=True, seed=42)
    base = list(one)
    r0, r1 = list(s[0]), list(s[1])
    assert len(r0) == len(r1) == 5
    for i in range(5):
        assert torch.equal(r0[i], base[2 * i]) and torch.equal(r1[i], base[2 * i + 1])
    s[0].set_epoch(1)
    assert not torch.equal(list(s[0])[0], r0[0])


def test_assistant_only_loss_masks_prompt():
    tk = load_tokenizer()
    rows = generate_qa(4, seed=3)
    ds = tokenize_rows(rows, tk, 1024, assistant_only_loss=True)
    b = C.SFTCollator(tk.pad_token_id)(ds, torch.tensor([0]))
    st = int(ds.loss_start[0])
    assert (b["labels"][0, :st] == -100).all() and (b["labels"][0, st:int(ds.lengths()[0])] != -100).all()


def _main_first_worker(rank, world, port, out_dir, forbid):
    import os
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import llm_fine_tune_distributed_amd.parallel.process_group as pgm
    pgm._STATE = None
    from llm_fine_tune_distributed_amd.data import dataset as dsm
    from llm_fine_tune_distributed_amd.data.synthetic import generate_qa
    from llm_fine_tune_distributed_amd.models import build_model, tiny
    from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer
    calls = []
    orig = dsm.tokenize_rows

    def spy(*a, **k):
        calls.append(rank)
        if forbid:
            raise AssertionError("tokenised although the cache holds this dataset")
        return orig(*a, **k)

    dsm.tokenize_rows = spy
    rows = [{"full-question": r["full-question"], "answer": r["answer"]} for r in generate_qa(24, seed=5)]
    args = SFTConfig(output_dir=out_dir, jsonl_log=False, max_steps=1, save_strategy="no",
                     dataset_cache=os.path.join(out_dir, "cache"))
    t = SFTTrainer(model=build_model(tiny(vocab_size=16384), dtype=torch.float32, seed=0), args=args,
                   train_dataset=rows)
    torch.save({"tokens": t.train_dataset.tokens, "offsets": t.train_dataset.offsets, "calls": calls,
                "vocab": t.tokenizer.vocab_size}, os.path.join(out_dir, f"tok{int(forbid)}_{rank}.pt"))
    pgm.cleanup_distributed()


def test_tokenisation_on_main_process_first_with_cache():
    """TRL main_process_first: rank 0 trains the tokenizer and tokenises, the other rank loads
    both behind a barrier; a second run with the same inputs loads the cached CSR arrays."""
    import os
    import socket
    import tempfile

    import torch
    import torch.multiprocessing as mp

    def port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    d = tempfile.mkdtemp()
    mp.spawn(_main_first_worker, args=(2, port(), d, False), nprocs=2, join=True)
    r0, r1 = (torch.load(os.path.join(d, f"tok0_{r}.pt")) for r in range(2))
    assert r0["calls"] == [0] and r1["calls"] == []  # only rank 0 tokenised
    assert torch.equal(r0["tokens"], r1["tokens"]) and torch.equal(r0["offsets"], r1["offsets"])
    assert r0["vocab"] == r1["vocab"]
    assert any(f.startswith("tokenized-") for f in os.listdir(os.path.join(d, "cache")))
    mp.spawn(_main_first_worker, args=(2, port(), d, True), nprocs=2, join=True)  # cache hit on every rank
    c0 = torch.load(os.path.join(d, "tok1_0.pt"))
    assert torch.equal(c0["tokens"], r0["tokens"])


def test_collator_max_batch_tokens_bounds_every_batch():
    """SFTCollator.max_batch_tokens is a hard bound of input_ids.numel() over every batch (padded, padding-free,
    explicit packing), derived from the data itself: the sparse tied-embedding gather size relies on it."""
    import torch
    from llm_fine_tune_distributed_amd.data.collator import SFTCollator
    from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset
    ds = TokenizedDataset.synthetic(40, 500, 3, 37, seed=11)
    g = torch.Generator().manual_seed(0)
    for col in (SFTCollator(0, 64, None, False), SFTCollator(0, 8, 16, False), SFTCollator(0, 256, None, True),
                SFTCollator(0, 1, None, True), SFTCollator(0, 16, 64, True, max_tokens=64)):
        for B in (1, 3, 7):
            cap = col.max_batch_tokens(ds, B)
            worst = 0
            for _ in range(30):
                idx = torch.randperm(len(ds), generator=g)[:B]
                worst = max(worst, col(ds, idx)["input_ids"].numel())
            assert 0 < worst <= cap, (col.__dict__, B, worst, cap)


def test_loader_producer_thread_ends_when_the_consumer_stops_early():
    """A consumer that stops mid-epoch (max_steps) closes the loader's generator: the collate thread parked on the
    full prefetch queue must exit instead of living on with its batches."""
    import threading
    ds = TokenizedDataset.synthetic(64, 1024, 16, 32, seed=0)
    dl = C.DataLoader(ds, C.SFTCollator(pad_token_id=0), C.DistributedBatchSampler(len(ds), 2, 1, 0, shuffle=False),
                      torch.device("cpu"), prefetch=1)
    it = dl.iter()
    next(it)
    assert any(t.name == "sftamd-collate" for t in threading.enumerate())
    it.close()
    assert not any(t.name == "sftamd-collate" and t.is_alive() for t in threading.enumerate())
    assert sum(1 for _ in dl) == len(dl)  # a full pass still sees every batch
