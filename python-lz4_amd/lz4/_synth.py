"""Deterministic synthetic corpora for tests and benchmarks.

The Silesia corpus named by the benchmark configuration is not available
offline, so ``silesia_like`` stands in for it: a seeded mix of 64 KiB blocks
of word text (Zipf vocabulary), C-like source, little-endian binary records,
random bytes and zero/byte runs.  The mix is tuned so that
``LZ4_compress_default`` reaches an aggregate ratio near the public Silesia
LZ4 ratio (~2.1).  It is a substitute, stated as such wherever it is used.

Everything here is plain numpy; nothing here compresses or decompresses.
"""
from __future__ import annotations

import numpy as np

BLOCK = 65536

_LETTERS = np.frombuffer(b"etaoinshrdlucmfwypvbgkjqxz", dtype=np.uint8)
_C_TOKENS = [
    b"int", b"return", b"if", b"else", b"for", b"while", b"static", b"const", b"void",
    b"char", b"unsigned", b"struct", b"size_t", b"uint32_t", b"NULL", b"sizeof", b"break",
    b"(", b")", b"{", b"}", b";", b"=", b"==", b"+", b"-", b"*", b"->", b"[", b"]", b",",
    b"0", b"1", b"i", b"j", b"n", b"len", b"buf", b"ptr", b"ctx", b"state", b"result",
    b"memcpy", b"printf", b"assert", b"<", b">", b"<=", b"&&", b"||", b"++",
]


def _vocab(rng: np.random.Generator, n_words: int, min_len: int = 1, max_len: int = 11):
    """A vocabulary as one byte buffer (each word followed by a space)."""
    lens = np.clip(rng.poisson(4.5, size=n_words) + 1, min_len, max_len)
    total = int(lens.sum() + n_words)
    probs = 1.0 / np.arange(1, _LETTERS.size + 1) ** 0.9
    probs /= probs.sum()
    letters = _LETTERS[rng.choice(_LETTERS.size, size=total, p=probs)]
    starts = np.concatenate([[0], np.cumsum(lens + 1)[:-1]])
    letters[starts + lens] = ord(" ")
    return letters, starts, lens + 1


def _emit_words(rng, buf, starts, lens, probs, n_bytes):
    """Concatenate Zipf-sampled words until n_bytes are produced."""
    mean_len = float((lens * probs).sum())
    k = int(n_bytes / mean_len * 1.2) + 16
    idx = rng.choice(starts.size, size=k, p=probs)
    wl = lens[idx]
    total = int(wl.sum())
    while total < n_bytes:
        more = rng.choice(starts.size, size=k, p=probs)
        idx = np.concatenate([idx, more])
        wl = lens[idx]
        total = int(wl.sum())
    offs = np.cumsum(wl) - wl
    src = np.repeat(starts[idx] - offs, wl) + np.arange(total)
    return buf[src][:n_bytes]


def word_text(rng: np.random.Generator, n_bytes: int) -> np.ndarray:
    buf, starts, lens = _vocab(rng, 6000)
    probs = 1.0 / (np.arange(starts.size) + 2.7) ** 1.07
    probs /= probs.sum()
    out = _emit_words(rng, buf, starts, lens, probs, n_bytes)
    spaces = np.flatnonzero(out == ord(" "))
    if spaces.size:
        nl = spaces[rng.random(spaces.size) < 0.06]
        out[nl] = ord("\n")
        cm = spaces[rng.random(spaces.size) < 0.05]
        out[np.maximum(cm - 1, 0)] = ord(",")
    return out


def c_source(rng: np.random.Generator, n_bytes: int) -> np.ndarray:
    toks = _C_TOKENS + [bytes(rng.choice(_LETTERS, size=int(rng.integers(3, 12)))) for _ in range(400)]
    chunks = [t + b" " for t in toks] + [b"\n    ", b"\n        ", b"\n}\n\n", b"\n"]
    buf = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy()
    lens = np.array([len(c) for c in chunks])
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    probs = 1.0 / (np.arange(len(chunks)) + 1.5) ** 0.95
    probs[-4:] = [0.05, 0.03, 0.005, 0.02]
    probs /= probs.sum()
    return _emit_words(rng, buf, starts, lens, probs, n_bytes)


def binary_records(rng: np.random.Generator, n_bytes: int) -> np.ndarray:
    """Little-endian 16-byte records: id, type, small delta timestamp, float random walk."""
    n = n_bytes // 16 + 1
    rec = np.zeros(n, dtype=[("id", "<u4"), ("kind", "<u2"), ("flags", "<u2"), ("ts", "<u4"), ("val", "<f4")])
    rec["id"] = np.arange(n, dtype=np.uint32) + np.uint32(rng.integers(0, 1 << 20))
    rec["kind"] = rng.choice(np.array([1, 2, 3, 7, 9], dtype=np.uint16), size=n)
    rec["flags"] = (rng.random(n) < 0.1).astype(np.uint16)
    rec["ts"] = np.cumsum(rng.integers(0, 40, size=n)).astype(np.uint32) + np.uint32(1_600_000_000)
    rec["val"] = np.round(np.cumsum(rng.normal(0, 1, size=n)), 1).astype(np.float32)
    return np.frombuffer(rec.tobytes(), dtype=np.uint8)[:n_bytes].copy()


def markup(rng: np.random.Generator, n_bytes: int) -> np.ndarray:
    """XML-like records: repetitive tags around short variable fields."""
    tags = [b"<entry id=\"", b"\">", b"<name>", b"</name>", b"<value unit=\"ms\">", b"</value>",
            b"<ref href=\"#", b"\"/>", b"</entry>\n", b"  "]
    names = [bytes(rng.choice(_LETTERS, size=int(rng.integers(4, 10)))) for _ in range(300)]
    parts, size, i = [], 0, int(rng.integers(0, 100000))
    while size < n_bytes:
        nm = names[int(min(rng.zipf(1.3), 300)) - 1]
        rec = b"".join([tags[9], tags[0], str(i).encode(), tags[1], tags[2], nm, tags[3], tags[4],
                        str(int(rng.integers(0, 999))).encode(), tags[5], tags[6],
                        str(i - int(rng.integers(1, 50))).encode(), tags[7], tags[8]])
        parts.append(rec)
        size += len(rec)
        i += 1
    return np.frombuffer(b"".join(parts), dtype=np.uint8)[:n_bytes].copy()


def random_bytes(rng: np.random.Generator, n_bytes: int) -> np.ndarray:
    return rng.integers(0, 256, size=n_bytes, dtype=np.uint8)


def runs(rng: np.random.Generator, n_bytes: int) -> np.ndarray:
    """Zero-dominated runs with occasional short random islands."""
    out = np.zeros(n_bytes, dtype=np.uint8)
    pos = 0
    while pos < n_bytes:
        run = int(rng.integers(64, 4096))
        pos += run
        isl = int(rng.integers(1, 48))
        end = min(n_bytes, pos + isl)
        if pos < n_bytes:
            out[pos:end] = rng.integers(0, 256, size=end - pos, dtype=np.uint8)
        pos = end
    return out


KINDS = {
    "text": word_text,
    "source": c_source,
    "records": binary_records,
    "markup": markup,
    "random": random_bytes,
    "runs": runs,
}
# block-kind mix of the Silesia substitute (fractions of blocks)
SILESIA_MIX = (("text", 0.34), ("source", 0.16), ("markup", 0.17), ("records", 0.20), ("random", 0.08),
               ("runs", 0.05))


def blocks(n_blocks: int, kind: str = "silesia", seed: int = 2026, block: int = BLOCK) -> np.ndarray:
    """``n_blocks`` x ``block`` uint8 array.

    ``kind`` is one of KINDS or ``"silesia"`` (the seeded mix).  Each block
    kind is generated as one contiguous stream and cut into blocks, so text
    blocks look like consecutive pages of one document.
    """
    rng = np.random.default_rng(seed)
    out = np.empty((n_blocks, block), dtype=np.uint8)
    if kind != "silesia":
        out[:] = KINDS[kind](rng, n_blocks * block).reshape(n_blocks, block)
        return out
    names = [k for k, _ in SILESIA_MIX]
    p = np.array([w for _, w in SILESIA_MIX])
    choice = rng.choice(len(names), size=n_blocks, p=p / p.sum())
    for ki, name in enumerate(names):
        sel = np.flatnonzero(choice == ki)
        if sel.size:
            out[sel] = KINDS[name](rng, sel.size * block).reshape(sel.size, block)
    return out
