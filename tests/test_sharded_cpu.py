"""CPU, world_size 2 (and 4) over gloo: the latent-sharded step orchestration (sharded.ShardedStep —
the same collectives and combine rules the GPU path uses) driven by a torch-CPU backend must
reproduce the unsharded oracle step."""
import os
import pathlib
import random
import signal

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from crosscoder_amd import sharded
from oracle import cpu_reference as O

B, N_MODELS, D, H, STEPS = 32, 2, 16, 64, 3


class CpuShardBackend:
    """Local compute of one latent shard with torch autograd (test-side stand-in for the GPU)."""

    def __init__(self, P, slices=2):
        self.P = {k: torch.nn.Parameter(v.detach().clone()) for k, v in P.items()}
        self.slices = slices
        self.m = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.rs = False
        self.row_align = 1

    def forward_partial(self, raw, factor):
        self.x = O.buffer_next(raw, factor)
        self.acts = torch.relu(torch.einsum("bnd,ndh->bh", self.x, self.P["W_enc"]) + self.P["b_enc"])
        self.partial = torch.einsum("bh,hnd->bnd", self.acts, self.P["W_dec"])
        self.recon = self.partial.detach().clone().contiguous()
        return self.recon

    def row_chunks(self):
        # several slices: the sliced (asynchronous) all-reduce; one: the synchronous one
        return [(i * B // self.slices, (i + 1) * B // self.slices) for i in range(self.slices)]

    def rows_ready(self, r0, r1, l1c):
        pass  # the torch backend does all loss / backward work in loss_finalize / backward

    def reduce_buffer(self):
        return torch.zeros(6)

    def loss_finalize(self, red):
        scalars = self.rs_scalars() if self.rs else self.loss_from_full_recon()
        red[4:6] = scalars[1:3]
        return scalars

    # ---- comm="reduce_scatter": loss on this rank's rows, then the gathered g_recon drives the backward
    def own_recon_buffer(self, rows):
        self.rs = True
        return torch.empty(rows, N_MODELS, D)

    def loss_own_rows(self, mine, r0, r1):
        with torch.no_grad():
            x = self.x
            diff = mine + self.P["b_dec"] - x[r0:r1]
            self.g_rows = (2.0 * diff / x.shape[0]).contiguous()
            l2_rows = diff.pow(2).sum(dim=(1, 2))
            tv_rows = (x[r0:r1] - x.mean(0)).pow(2).sum(dim=(1, 2))
            self.terms = torch.stack([l2_rows, 1 - l2_rows / (tv_rows + 1e-8)])
            self.dbd = self.g_rows.sum(0, keepdim=True)

    def gather_pairs(self, r0, r1, world):
        B = self.x.shape[0]
        self.g_full = torch.empty(B, N_MODELS, D)
        self.terms_all = torch.empty(world * 2, r1 - r0)  # (concatenated along dim 0: gloo's form)
        self.dbd_all = torch.empty(world, N_MODELS, D)
        return [(self.g_full, self.g_rows), (self.terms_all, self.terms), (self.dbd_all, self.dbd)]

    def after_gather(self, l1c):
        self.l1 = (self.acts * self.P["W_dec"].norm(dim=-1).sum(1)[None]).sum(-1).mean(0)

    def rs_scalars(self):
        t = self.terms_all.view(-1, 2, self.terms_all.shape[1]).permute(1, 0, 2).reshape(2, -1)
        l0 = (self.acts > 0).float().sum(-1).mean()
        ev = t[1].mean()
        return torch.stack([t[0].mean(), self.l1.detach(), l0, ev, ev, ev])

    def loss_from_full_recon(self):
        self.R = self.recon.clone().requires_grad_(True)
        full = self.R + self.P["b_dec"]
        x = self.x
        l2_row = (full - x).pow(2).sum(dim=(1, 2))
        self.l2 = l2_row.mean()
        tv = (x - x.mean(0)).pow(2).sum(dim=(1, 2))
        ev = 1 - l2_row / (tv + 1e-8)
        tn = self.P["W_dec"].norm(dim=-1).sum(1)
        self.l1 = (self.acts * tn[None]).sum(-1).mean(0)
        l0 = (self.acts > 0).float().sum(-1).mean()
        return torch.stack([self.l2.detach(), self.l1.detach(), l0, ev.mean().detach(), ev.mean().detach(),
                            ev.mean().detach()])

    def backward(self, l1c, red, rank):
        for p in self.P.values():
            p.grad = None
        if self.rs:  # d(l2)/d(recon) = the gathered g_recon; d(l2)/d(b_dec) = the ranks' row sums
            (self.partial * self.g_full).sum().add(l1c * self.l1).backward()
            self.P["b_dec"].grad = self.dbd_all.sum(0)
        else:
            gl2 = torch.autograd.grad(self.l2, [self.R, self.P["b_dec"]], retain_graph=True)
            (self.partial * gl2[0]).sum().add(l1c * self.l1).backward()
            self.P["b_dec"].grad = gl2[1]
        sums = torch.stack([self.P[k].grad.pow(2).sum() for k in O.PARAM_ORDER])
        red[0:4] = sharded.clip_sums_for_allreduce(sums, rank)

    def clip_and_adam_from_sums(self, sums, lr, betas, eps, t, max_norm):
        total = sums.sqrt().norm()
        coef = min(1.0, max_norm / (total.item() + 1e-6))
        with torch.no_grad():
            for k in O.PARAM_ORDER:
                g = self.P[k].grad * coef
                O.adam_update(self.P[k].data, g, self.m[k], self.v[k], float(t), lr, betas[0], betas[1], eps)


def _setup():
    cfg = {"seed": 49, "dict_size": H, "d_in": D, "enc_dtype": "fp32", "dec_init_norm": 0.08, "batch_size": B,
           "num_tokens": B * 10, "lr": 1e-3, "beta1": 0.9, "beta2": 0.999, "l1_coeff": 2}
    P = O.init_params(cfg)
    g = torch.Generator().manual_seed(0)
    raws = [torch.randn(B, N_MODELS, D, generator=g) * 3 for _ in range(STEPS)]
    factor = torch.tensor([0.5, 0.25])
    return cfg, P, raws, factor


def _worker(rank, world, port, q, comm, slices=2):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, P, raws, factor = _setup()
        lo, hi = sharded.shard_range(H, world, rank)
        Ps = {"W_enc": P["W_enc"][:, :, lo:hi], "W_dec": P["W_dec"][lo:hi], "b_enc": P["b_enc"][lo:hi],
              "b_dec": P["b_dec"]}
        backend = CpuShardBackend(Ps, slices)
        step = sharded.ShardedStep(backend, comm=comm)
        outs = []
        seen = []

        def on_losses(scalars, red):
            # called after the all-reduce of the sums and l1 / l0, before the clip / Adam
            seen.append(red.clone())

        for t in range(STEPS):
            l1c = 2.0 if t else 0.0
            cb = on_losses if t % 2 else None
            s, red = step.step(raws[t], factor, l1c, cfg["lr"], (0.9, 0.999), 1e-8, t + 1, on_losses=cb)
            if cb is not None:
                assert torch.equal(seen[-1], red)
            outs.append(torch.stack([s[0], red[4], red[5]]).clone())
        # numpy arrays pickle by value: a torch tensor would travel as a shared-memory fd that the
        # parent can only open while this process is still alive
        q.put((rank, [o.tolist() for o in outs], {k: v.detach().numpy().copy() for k, v in backend.P.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm,slices", [("all_reduce", 2), ("all_reduce", 4), ("all_reduce", 1), ("reduce_scatter", 1)])
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_step_matches_unsharded(world, comm, slices):
    """Both exchanges of the partial reconstructions: the all-reduce (in two or four batch slices,
    or one synchronous collective), and the reduce-scatter by batch rows -> loss on B/G rows -> all-gather
    of g_recon and the row terms."""
    port = 29500 + random.randint(0, 2000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, comm, slices)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, outs, Pl = q.get(timeout=300)
        res[r] = (outs, Pl)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    cfg, P, raws, factor = _setup()
    ref = {k: torch.nn.Parameter(v.detach().clone()) for k, v in P.items()}
    m = {k: torch.zeros_like(v) for k, v in ref.items()}
    v = {k: torch.zeros_like(v) for k, v in ref.items()}
    for t in range(STEPS):
        l1c = 2.0 if t else 0.0
        x = O.buffer_next(raws[t], factor)
        lo = O.get_losses(x, ref, torch.float32)
        for p in ref.values():
            p.grad = None
        (lo["l2_loss"] + l1c * lo["l1_loss"]).backward()
        with torch.no_grad():
            O.clip_grad_norm([ref[k].grad for k in O.PARAM_ORDER])
            for k in O.PARAM_ORDER:
                O.adam_update(ref[k].data, ref[k].grad, m[k], v[k], float(t + 1), cfg["lr"], 0.9, 0.999, 1e-8)
        for r in range(world):
            l2, l1, l0 = res[r][0][t]
            assert abs(l2 - lo["l2_loss"].item()) <= 1e-5 * abs(lo["l2_loss"].item())
            assert abs(l1 - lo["l1_loss"].item()) <= 1e-5 * abs(lo["l1_loss"].item()) + 1e-7
            assert abs(l0 - lo["l0_loss"].item()) <= 1e-6
    for r in range(world):
        lo_, hi_ = sharded.shard_range(H, world, r)
        Pl = {k: torch.from_numpy(a) for k, a in res[r][1].items()}
        torch.testing.assert_close(Pl["W_dec"], ref["W_dec"].detach()[lo_:hi_], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(Pl["W_enc"], ref["W_enc"].detach()[:, :, lo_:hi_], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(Pl["b_enc"], ref["b_enc"].detach()[lo_:hi_], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(Pl["b_dec"], ref["b_dec"].detach(), rtol=1e-5, atol=1e-6)


def test_shard_range_and_clip_combine():
    assert sharded.shard_range(131072, 8, 3) == (49152, 65536)
    with pytest.raises(ValueError):
        sharded.shard_range(100, 8, 0)
    s = torch.tensor([1.0, 2.0, 3.0, 4.0])
    assert sharded.clip_sums_for_allreduce(s, 0).tolist() == [1, 2, 3, 4]
    assert sharded.clip_sums_for_allreduce(s, 1).tolist() == [1, 2, 3, 0]


def _init_worker(rank, world, port, q, enc_dtype, tmpdir, d_in):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import crosscoder_amd as ca
        from crosscoder_amd import crosscoder as ccmod

        cfg = {"seed": 49, "dict_size": 96, "d_in": d_in, "enc_dtype": enc_dtype, "dec_init_norm": 0.08,
               "device": "cpu"}
        lo, hi = sharded.shard_range(cfg["dict_size"], world, rank)
        cc = sharded.shard_crosscoder(cfg, lo, hi)
        full = ca.CrossCoder(cfg)
        # this rank's slice IS the reference init of the whole dictionary, sliced
        assert torch.equal(cc.W_dec.detach(), full.W_dec.detach()[lo:hi])
        assert torch.equal(cc.W_enc.detach(), full.W_enc.detach()[:, :, lo:hi])
        sd = sharded.gather_state_dict(cc, cfg["dict_size"])
        ref = full.reference_state_dict()
        assert list(sd) == list(ref)
        for k in ref:
            assert torch.equal(sd[k], ref[k]) and sd[k].stride() == ref[k].stride(), k
        # the checkpoint path: gathered on rank 0 only (host tensors), the same dict
        sd0 = sharded.gather_state_dict(cc, cfg["dict_size"], dst=0)
        if rank == 0:
            assert list(sd0) == list(ref)
            for k in ref:
                assert sd0[k].device.type == "cpu"
                assert torch.equal(sd0[k], ref[k]) and sd0[k].stride() == ref[k].stride(), k
            ccmod.write_checkpoint(sd0, cfg, save_dir=pathlib.Path(tmpdir), version=0)
        else:
            assert sd0 is None
        dist.barrier()
        q.put((rank, True))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("enc_dtype,d_in", [("fp32", 24), ("bf16", 24), ("bf16", 20)])
def test_sharded_init_is_reference_slice_and_gathers_back(enc_dtype, d_in, tmp_path):
    """ShardedTrainer's default init (shard_crosscoder) gives rank r latents [lo, hi) of exactly the
    crosscoder the reference builds for the whole dictionary (crosscoder.py:31-62), and
    gather_state_dict reassembles the reference state_dict (values, key order, W_enc strides); the
    rank-0 checkpoint is the reference's two-file format (crosscoder.py:132-146)."""
    world = 2
    port = 29500 + random.randint(2001, 4000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_init_worker, args=(r, world, port, q, enc_dtype, str(tmp_path), d_in)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: True, 1: True}
    import json

    import crosscoder_amd as ca

    cfg = json.load(open(tmp_path / "0_cfg.json"))
    sd = torch.load(tmp_path / "0.pt", weights_only=True)
    ref = ca.CrossCoder(cfg).reference_state_dict()
    for k in ref:
        assert torch.equal(sd[k], ref[k]) and sd[k].stride() == ref[k].stride(), k


class _Loop:
    """ShardedTrainer.train's collaborators (step / log / save / agree_stop), counted."""
    total_steps = 8
    cfg = {"log_every": 100, "save_every": 1000, "stop_check_every": 2}

    def __init__(self, fail_at=None, exc=None, group=None):
        self.n, self.saved, self.fail_at, self.exc, self.group = 0, 0, fail_at, exc, group

    def step(self):
        self.n += 1
        if self.n == self.fail_at:
            if self.exc is None:
                os.kill(os.getpid(), signal.SIGINT)  # (the handler train() installed only sets a flag)
            else:
                raise self.exc()
        return {}

    def log(self, d):
        pass

    def save(self):
        self.saved += 1

    def agree_stop(self, flag):
        return sharded.agree_stop(flag, self.group) if self.group is not None else flag


def test_sharded_train_final_save_on_interrupt_only():
    """ShardedTrainer.train keeps the reference's final save (trainer.py:81-82) where every rank leaves the loop
    at the same step: normal completion, and SIGINT -- which only sets a flag the ranks agree on at the next
    `stop_check_every` step boundary (never a collective save started from inside a step's
    collectives) -- after which KeyboardInterrupt is raised.  Another exception, which may be one rank's alone,
    propagates without the collective save.  The SIGINT handler is restored afterwards."""
    prev = signal.getsignal(signal.SIGINT)
    done = _Loop()
    sharded.ShardedTrainer.train(done)
    assert (done.n, done.saved) == (8, 1)
    interrupted = _Loop(fail_at=3)
    with pytest.raises(KeyboardInterrupt):
        sharded.ShardedTrainer.train(interrupted)
    assert (interrupted.n, interrupted.saved) == (4, 1)  # (the step in flight and the next one finish first)
    failed = _Loop(fail_at=3, exc=RuntimeError)
    with pytest.raises(RuntimeError):
        sharded.ShardedTrainer.train(failed)
    assert failed.saved == 0
    assert signal.getsignal(signal.SIGINT) is prev


def _interrupt_rank(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        loop = _Loop(fail_at=3 if rank == 0 else None, group=None)
        loop.group = dist.group.WORLD
        try:
            sharded.ShardedTrainer.train(loop)
            q.put((rank, loop.n, loop.saved, "done"))
        except KeyboardInterrupt:
            q.put((rank, loop.n, loop.saved, "interrupt"))
    finally:
        dist.destroy_process_group()


def test_sharded_train_sigint_on_one_rank_stops_all_ranks_at_one_step():
    """World 2 over gloo: SIGINT reaches rank 0 only, during its step 3; both ranks leave the loop after step 4
    (the next agreement point), both run the final save and both raise KeyboardInterrupt."""
    world = 2
    port = 29000 + random.randint(0, 900)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_interrupt_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, 4, 1, "interrupt"), (1, 4, 1, "interrupt")]


# ----------------------------------------------------------------------------- one buffer for the whole group
def _torch_gather(src, perm, out=None):
    # (the tests of the group logic run the buffer on the CPU: torch indexing in place of cc_gather_rows)
    out = torch.empty_like(src) if out is None else out
    out.copy_(src[perm])
    return out


class _NoisyLM:
    """The golden fake LM (table[token] + pos), plus `noise` x a rank-dependent offset: a stand-in for LM
    forwards that are not bit-identical across ranks."""

    class _C:
        pass

    def __init__(self, table, pos, noise=0.0):
        self.table, self.pos, self.noise = table, pos, noise
        self.cfg = _NoisyLM._C()
        self.cfg.d_model = table.shape[1]

    def run_with_cache(self, tokens, names_filter=None, return_type=None):
        a = self.table[tokens] + self.pos[None, : tokens.shape[1]]
        if self.noise:
            a = a + self.noise * (1 + dist.get_rank())
        return None, {names_filter: a}


def _buffer_worker(rank, world, port, q, grouped, noise):
    import json

    import crosscoder_amd as ca

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = torch.load(os.path.join(os.path.dirname(__file__), "golden", "buffer_fake_lm.pt"), weights_only=True)
        cfg = json.loads(r["cfg"])
        ca.Buffer.gather_rows = staticmethod(_torch_gather)
        # rank 0 draws the reference's permutations (seed 49, as the fixture); the other ranks' generators differ
        torch.manual_seed(49 + 1000 * rank)
        lms = [_NoisyLM(r[f"{m}_table"], r[f"{m}_pos"], noise) for m in ("A", "B")]
        buf = ca.Buffer(cfg, *lms, r["tokens"], group=dist.group.WORLD if grouped else None)
        batches, errors = [], []

        class _T:  # ShardedTrainer's collaborators of _verify_buffer
            buffer, group, _verified = buf, None, None

        for _ in range(len(r["next"])):
            try:
                sharded.ShardedTrainer._verify_buffer(_T)
            except RuntimeError as e:
                errors.append(str(e))
                _T._verified = buf.refresh_count
            batches.append(buf.next().numpy().copy())
        q.put((rank, batches, buf.normalisation_factor.numpy().copy(), buf.refresh_count, errors))
    finally:
        dist.destroy_process_group()


def _run_buffer_ranks(world, grouped, noise):
    port = 28000 + random.randint(0, 900)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_buffer_worker, args=(r, world, port, q, grouped, noise)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rk, batches, factor, refreshes, errors = q.get(timeout=300)
        res[rk] = (batches, factor, refreshes, errors)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_grouped_buffer_equals_reference_buffer_on_every_rank(world):
    """Buffer(group=...) (SURVEY 8e "replicate x"): each rank harvests a contiguous share of the LM batches and the
    norm-estimate batches, the shares are broadcast, the permutation is drawn on rank 0 (torch's global CPU
    generator, as buffer.py:111-113) and broadcast.  Every rank's normalisation factors and every next() batch,
    across two refreshes, equal the reference Buffer's own outputs (tests/golden/buffer_fake_lm.pt, made by running
    the reference), although the ranks' CPU generators differ; the fingerprint check passes at every refresh."""
    r = torch.load(os.path.join(os.path.dirname(__file__), "golden", "buffer_fake_lm.pt"), weights_only=True)
    res = _run_buffer_ranks(world, grouped=True, noise=0.0)
    for rk in range(world):
        batches, factor, refreshes, errors = res[rk]
        assert errors == [] and refreshes >= 3
        assert torch.equal(torch.from_numpy(factor), r["normalisation_factor"])
        for got, want in zip(batches, r["next"]):
            assert torch.equal(torch.from_numpy(got), want)


def test_fingerprint_check_fires_when_ranks_harvest_alone():
    """LM forwards that differ across ranks (a rank-dependent offset): with every rank harvesting on its own (the
    reference Buffer per rank, group=None) the ranks' buffers differ and ShardedTrainer's fingerprint check raises
    on every rank at every buffer state; with group=... the ranks share one harvest, their batches are identical and
    the check passes."""
    alone = _run_buffer_ranks(2, grouped=False, noise=1e-3)
    for rk in range(2):
        batches, _, refreshes, errors = alone[rk]
        # (every buffer state a batch was taken from: the last refresh, by the last next(), served none)
        assert len(errors) == refreshes - 1 and all("buffers differ" in e for e in errors), errors
    assert not all(torch.equal(torch.from_numpy(a), torch.from_numpy(b)) for a, b in zip(alone[0][0], alone[1][0]))
    shared = _run_buffer_ranks(2, grouped=True, noise=1e-3)
    assert shared[0][3] == [] and shared[1][3] == []
    for a, b in zip(shared[0][0], shared[1][0]):
        assert torch.equal(torch.from_numpy(a), torch.from_numpy(b))


def test_sigint_after_the_last_stop_check_still_stops_all_ranks():
    """a SIGINT that arrives after the last `stop_check_every` boundary (total_steps not a multiple of
    it) is not dropped: the ranks agree once more after the loop, save and raise KeyboardInterrupt."""

    class _Odd(_Loop):
        total_steps = 7

    prev = signal.getsignal(signal.SIGINT)
    late = _Odd(fail_at=7)
    with pytest.raises(KeyboardInterrupt):
        sharded.ShardedTrainer.train(late)
    assert (late.n, late.saved) == (7, 1)
    assert signal.getsignal(signal.SIGINT) is prev
