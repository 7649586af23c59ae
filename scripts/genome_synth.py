"""Repeat-rich synthetic genomes for config C4 (GRCh38 itself is not in the
container and cannot be fetched).  Benchmark input only: the
counter never sees how the sequence was made.

A record is a run of segments drawn on the host (numpy, seeded) and expanded on
the device (torch):
  * unique sequence (uniform iid ACGT), lengths geometric around 1.5 kb;
  * interspersed repeats, ~45 % of the bases: copies of one of `families` repeat
    consensus sequences (300 bp - 6 kb; popularity Zipf-like, so a few families
    are very common, like Alu / L1), a random sub-interval of it, reverse
    complemented half of the time, with 0 - 15 % of the bases substituted
    (divergence skewed low: young, near-identical copies are common);
  * tandem repeats, ~3 %: a 1 - 60 bp unit repeated to 20 bp - 5 kb
    (homopolymers and microsatellites among them), lightly mutated;
  * N runs (~3 % of the bases) and soft-masking: repeat-derived bases lowercase
    (as RepeatMasker output is), so KMC_CANON_SOFTMASK counts them.
The repeats make many windows share a canonical key (reverse-complemented copies
fold onto the same keys), which exercises the counter's repeat path: the LDS
table's add for an already-claimed key, hot keys in a pass, long lists.
"""
import numpy as np

# relative sizes of chr1..22, X, Y, M-ish (both genomes below)
REL = [248, 242, 198, 190, 181, 171, 159, 145, 138, 134, 135, 133, 114, 107, 102, 90, 83, 80, 59, 64, 47, 51,
       156, 57, 1]

COMP = np.frombuffer(b"TGCA", dtype=np.uint8)  # complement of codes 0..3 (A C G T)


def _segments(rng, total, fam_len, fam_p, frac_rep=0.45, frac_tandem=0.03, frac_n=0.03):
    """Host plan of one record: arrays (length, kind, src, period, rc, mut); kind
    0 = unique, 1 = repeat copy (src = offset in the family pool), 2 = tandem
    (src = offset of its unit in the unit pool), 3 = N run."""
    fam_off = np.concatenate([[0], np.cumsum(fam_len)[:-1]])
    est = int(total / 600) + 64
    kinds = rng.choice(4, size=est, p=[1 - frac_rep - frac_tandem - frac_n, frac_rep, frac_tandem, frac_n])
    L = np.zeros(est, np.int64)
    src = np.zeros(est, np.int64)
    per = np.zeros(est, np.int64)
    rc = np.zeros(est, np.uint8)
    mut = np.zeros(est, np.float32)
    # unique: geometric around 1.5 kb
    m = kinds == 0
    L[m] = rng.geometric(1 / 1500, size=m.sum())
    # repeat copies: family by popularity, a sub-interval of it
    m = kinds == 1
    f = rng.choice(len(fam_len), size=m.sum(), p=fam_p)
    flen = fam_len[f]
    a = (rng.random(m.sum()) * flen * 0.5).astype(np.int64)
    b = flen - (rng.random(m.sum()) * (flen - a) * 0.3).astype(np.int64)
    L[m] = np.maximum(b - a, 20)
    src[m] = fam_off[f] + a
    per[m] = 0
    rc[m] = rng.random(m.sum()) < 0.5
    mut[m] = 0.15 * rng.random(m.sum()) ** 2  # divergence 0 - 15 %, young (close) copies common
    # tandem: unit 1..60 bp (short units common), 20 bp .. 5 kb long
    m = kinds == 2
    u = np.minimum(rng.geometric(0.25, size=m.sum()), 60)
    per[m] = u
    src[m] = rng.integers(0, 1 << 20, size=m.sum())  # offset in the unit pool
    L[m] = np.minimum(rng.geometric(1 / 300, size=m.sum()) + 20, 5000)
    mut[m] = rng.uniform(0.0, 0.03, size=m.sum())
    # N runs
    m = kinds == 3
    L[m] = rng.geometric(1 / 1000, size=m.sum())
    cs = np.cumsum(L)
    n = int(np.searchsorted(cs, total)) + 1
    if n > est:
        raise RuntimeError("segment plan too short")
    L = L[:n].copy()
    L[-1] -= cs[n - 1] - total
    return L, kinds[:n], src[:n], per[:n], rc[:n], mut[:n]


def repeat_genome(torch, dev, gbases, seed=38, families=3000, min_len=1000):
    """(data uint8 device tensor, indices int64 device tensor, record lengths,
    stats dict): chromosome-like records totalling gbases * 1e9 bases, each
    followed by '\\0'."""
    rng = np.random.default_rng(seed)
    tot = sum(REL)
    lens = [max(min_len, int(gbases * 1e9 * r / tot)) for r in REL]
    fam_len = rng.integers(300, 6001, size=families)
    zipf = 1.0 / np.arange(1, families + 1) ** 1.1
    fam_p = zipf / zipf.sum()
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    pool = torch.randint(0, 4, (int(fam_len.sum()),), device=dev, generator=g, dtype=torch.int64).to(torch.uint8)
    units = torch.randint(0, 4, ((1 << 20) + 64,), device=dev, generator=g, dtype=torch.int64).to(torch.uint8)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    comp = torch.tensor([3, 2, 1, 0], dtype=torch.uint8, device=dev)
    nbytes = sum(L + 1 for L in lens)
    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    off = 0
    stats = {"bases": 0, "repeat": 0, "tandem": 0, "n": 0}
    for L in lens:
        segL, kinds, src, per, rc, mut = _segments(rng, L, fam_len, fam_p)
        starts = np.concatenate([[0], np.cumsum(segL)[:-1]])
        for kname, kv in (("repeat", 1), ("tandem", 2), ("n", 3)):
            stats[kname] += int(segL[kinds == kv].sum())
        stats["bases"] += L
        t_start = torch.from_numpy(starts).to(dev)
        t_len = torch.from_numpy(segL).to(dev)
        t_kind = torch.from_numpy(kinds.astype(np.uint8)).to(dev)
        t_src = torch.from_numpy(src).to(dev)
        t_per = torch.from_numpy(per).to(dev)
        t_rc = torch.from_numpy(rc).to(dev)
        t_mut = torch.from_numpy(mut).to(dev)
        step = 1 << 27
        for c0 in range(0, L, step):
            c1 = min(L, c0 + step)
            pos = torch.arange(c0, c1, device=dev, dtype=torch.int64)
            s = torch.searchsorted(t_start, pos, right=True) - 1
            o = pos - t_start[s]
            kind = t_kind[s]
            code = torch.randint(0, 4, (c1 - c0,), device=dev, generator=g, dtype=torch.int64).to(torch.uint8)
            # repeat copies (reverse complement: read the family backwards, complemented)
            rep = kind == 1
            ln = t_len[s]
            rcm = t_rc[s].bool()
            fo = torch.where(rcm, ln - 1 - o, o)
            fam_code = pool[torch.clamp(t_src[s] + fo, max=pool.numel() - 1)]
            fam_code = torch.where(rcm, comp[fam_code.long()], fam_code)
            # tandem: unit base o mod period
            tan = kind == 2
            pr = torch.clamp(t_per[s], min=1)
            tan_code = units[(t_src[s] + o % pr).clamp(max=units.numel() - 1)]
            mutate = torch.rand(c1 - c0, device=dev, generator=g) < t_mut[s]
            code = torch.where(rep & ~mutate, fam_code, code)
            code = torch.where(tan & ~mutate, tan_code, code)
            b = lut[code.long()]
            b = torch.where(rep | tan, b | 0x20, b)  # soft-masked repeats
            b = torch.where(kind == 3, torch.full_like(b, ord("N")), b)
            data[off + c0:off + c1] = b
            del pos, s, o, kind, code, rep, ln, rcm, fo, fam_code, tan, pr, tan_code, mutate, b
        data[off + L] = 0
        off += L + 1
    idx = np.concatenate([[0], np.cumsum([L + 1 for L in lens])]).astype(np.int64)
    return data, torch.from_numpy(idx).to(dev), lens, stats


def grch38_like(torch, dev, gbases, seed=38):
    """Synthetic stand-in for GRCh38 (not in the container): chromosome-like
    record lengths, uniform bases, N runs and lowercase runs."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    rel = REL
    tot = sum(rel)
    lens = [max(1000, int(gbases * 1e9 * r / tot)) for r in rel]
    n = len(lens)
    nbytes = sum(L + 1 for L in lens)
    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    chunk = 1 << 28
    for o in range(0, nbytes, chunk):
        m = min(chunk, nbytes - o)
        data[o:o + m] = lut[torch.randint(0, 4, (m,), device=dev, generator=g, dtype=torch.int64).to(torch.uint8).long()]
        # runs of 4096 bases: ~50 % lowercase, ~5 % N
        r = torch.rand((m + 4095) // 4096, device=dev, generator=g)
        run = r.repeat_interleave(4096)[:m]
        seg = data[o:o + m]
        seg[run < 0.5] += 32
        seg[run > 0.95] = ord("N")
    off = [0]
    for L in lens:
        off.append(off[-1] + L + 1)
    offs = torch.tensor(off, dtype=torch.int64)
    data[offs[1:] - 1] = 0
    return data, offs.to(dev), lens
