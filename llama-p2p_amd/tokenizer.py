"""Tokenizer / detokenizer built from GGUF metadata.

The reference tokenizes inside ``self.model(prompt, max_tokens=100)``
(/root/reference/llama_p2p_network.py:125): llama-cpp-python calls
``Llama.tokenize(prompt.encode(), add_bos=True, special=True)`` and
``Llama.detokenize`` on the completion.  Both are llama.cpp's vocab code,
restated here from the GGUF keys a model file carries:

* ``tokenizer.ggml.model == "llama"`` -> SentencePiece BPE (llm_tokenizer_spm):
  add a leading space, spaces -> U+2581, split into UTF-8 characters, repeatedly
  merge the adjacent pair whose concatenation is a vocab piece with the highest
  score (leftmost on ties), then unknown pieces fall back to ``<0xXX>`` byte tokens.
* ``tokenizer.ggml.model == "gpt2"`` -> byte-level BPE (llm_tokenizer_bpe) with
  the Llama-3 pre-tokenizer regex and ``tokenizer.ggml.merges`` ranks.

Host-side only: tokenization is negligible next to the forward pass.
"""
from __future__ import annotations

import heapq
import re
from typing import Dict, List, Optional, Sequence

SPACE = "▁"
_SPM_SEGMENT = re.compile(SPACE + "+[^" + SPACE + "]*|[^" + SPACE + "]+")  # split before SPACE after non-SPACE
TOKEN_NORMAL, TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_USER, TOKEN_UNUSED, TOKEN_BYTE = 1, 2, 3, 4, 5, 6

LLAMA3_PRETOKENIZE = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|"
                      r"\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")


def _bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


class Tokenizer:
    def __init__(self, tokens: Sequence[str], scores: Optional[Sequence[float]] = None,
                 types: Optional[Sequence[int]] = None, model: str = "llama", merges: Optional[Sequence[str]] = None,
                 bos_id: int = 1, eos_id: int = 2, unk_id: int = 0, add_bos: bool = True,
                 add_space_prefix: bool = True, eot_id: Optional[int] = None):
        self.tokens = list(tokens)
        self.n_vocab = len(self.tokens)
        self.scores = list(scores) if scores is not None else [0.0] * self.n_vocab
        self.types = list(types) if types is not None else [TOKEN_NORMAL] * self.n_vocab
        self.model = model
        self.bos_id, self.eos_id, self.unk_id, self.eot_id = bos_id, eos_id, unk_id, eot_id
        self.add_bos = add_bos
        self.add_space_prefix = add_space_prefix
        self.piece_to_id: Dict[str, int] = {}
        for i, t in enumerate(self.tokens):
            self.piece_to_id.setdefault(t, i)
        self.byte_ids: Dict[int, int] = {}
        for i, (t, ty) in enumerate(zip(self.tokens, self.types)):
            if ty == TOKEN_BYTE and len(t) == 6 and t.startswith("<0x"):
                self.byte_ids[int(t[3:5], 16)] = i
        self.special = {t: i for i, (t, ty) in enumerate(zip(self.tokens, self.types))
                        if ty in (TOKEN_CONTROL, TOKEN_USER)}
        self.bpe_ranks: Dict[tuple, int] = {}
        if merges:
            for r, m in enumerate(merges):
                a, _, b = m.partition(" ")
                self.bpe_ranks[(a, b)] = r
        self._b2u = _bytes_to_unicode()
        self._u2b = {v: k for k, v in self._b2u.items()}
        self._re = None
        # SPM text splits exactly at every SPACE that follows a non-SPACE character when no vocabulary
        # piece holds such a pair (merges never cross those boundaries), and BPE works per regex word:
        # both tokenise repeated segments once (per-segment cache; llama.cpp tokenises in C++)
        self._spm_split = not any(SPACE in t[1:] and any(t[i] == SPACE and t[i - 1] != SPACE for i in range(1, len(t)))
                                  for t in self.tokens)
        self._seg_cache: Dict[str, List[int]] = {}

    # ------------------------------------------------------------------ load
    @classmethod
    def from_gguf_metadata(cls, md: dict) -> "Tokenizer":
        model = md.get("tokenizer.ggml.model", "llama")
        toks = md.get("tokenizer.ggml.tokens")
        if not toks:
            raise ValueError("GGUF has no tokenizer.ggml.tokens")
        return cls(toks, md.get("tokenizer.ggml.scores"), md.get("tokenizer.ggml.token_type"), model,
                   md.get("tokenizer.ggml.merges"), int(md.get("tokenizer.ggml.bos_token_id", 1)),
                   int(md.get("tokenizer.ggml.eos_token_id", 2)), int(md.get("tokenizer.ggml.unknown_token_id", 0)),
                   bool(md.get("tokenizer.ggml.add_bos_token", True)),
                   bool(md.get("tokenizer.ggml.add_space_prefix", model == "llama")),
                   md.get("tokenizer.ggml.eot_token_id"))

    # ------------------------------------------------------------- tokenize
    def tokenize(self, text: bytes, add_bos: bool = True, special: bool = False) -> List[int]:
        s = text.decode("utf-8", errors="replace") if isinstance(text, (bytes, bytearray)) else str(text)
        out: List[int] = [self.bos_id] if (add_bos and self.add_bos) else []
        first = True
        for frag, sid in self._split_special(s, special):
            if sid is not None:
                out.append(sid)
                continue
            if self.model == "gpt2":
                out.extend(self._bpe(frag))
            else:
                if self.add_space_prefix and first:
                    frag = " " + frag
                out.extend(self._spm(frag))
            first = False
        return out

    def _split_special(self, s: str, special: bool):
        if not special or not self.special or not s:
            return [(s, None)] if s else []
        parts = [(s, None)]
        for tok in sorted(self.special, key=len, reverse=True):
            nxt = []
            for frag, sid in parts:
                if sid is not None or tok not in frag:
                    nxt.append((frag, sid))
                    continue
                pieces = frag.split(tok)
                for j, p in enumerate(pieces):
                    if p:
                        nxt.append((p, None))
                    if j + 1 < len(pieces):
                        nxt.append((tok, self.special[tok]))
            parts = nxt
        return parts

    def _cached(self, seg: str, fn) -> List[int]:
        ids = self._seg_cache.get(seg)
        if ids is None:
            if len(self._seg_cache) > 200000:
                self._seg_cache.clear()
            ids = self._seg_cache[seg] = fn(seg)
        return ids

    def _spm(self, text: str) -> List[int]:
        text = text.replace(" ", SPACE)
        if not text:
            return []
        if not self._spm_split:
            return self._spm_seg(text)
        out: List[int] = []
        for m in _SPM_SEGMENT.finditer(text):
            out.extend(self._cached(m.group(0), self._spm_seg))
        return out

    def _spm_seg(self, text: str) -> List[int]:
        sym = list(text)  # UTF-8 characters
        n = len(sym)
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        nxt[-1] = -1
        alive = [True] * n
        heap = []

        def push(l, r):
            if l < 0 or r < 0:
                return
            pid = self.piece_to_id.get(sym[l] + sym[r])
            if pid is None:
                return
            heapq.heappush(heap, (-self.scores[pid], l, r, sym[l] + sym[r]))

        for i in range(n - 1):
            push(i, i + 1)
        while heap:
            _, l, r, txt = heapq.heappop(heap)
            if not alive[l] or not alive[r] or nxt[l] != r or sym[l] + sym[r] != txt:
                continue
            sym[l] = txt
            alive[r] = False
            nxt[l] = nxt[r]
            if nxt[r] >= 0:
                prev[nxt[r]] = l
            push(prev[l], l)
            push(l, nxt[l])
        out = []
        i = 0
        while i >= 0 and i < n:
            if alive[i]:
                pid = self.piece_to_id.get(sym[i])
                if pid is not None:
                    out.append(pid)
                else:
                    for b in sym[i].encode("utf-8"):
                        out.append(self.byte_ids.get(b, self.unk_id))
            i = nxt[i]
        return out

    def _bpe(self, text: str) -> List[int]:
        if self._re is None:
            import regex

            self._re = regex.compile(LLAMA3_PRETOKENIZE)
        out = []
        for word in self._re.findall(text):
            out.extend(self._cached(word, self._bpe_word))
        return out

    def _bpe_word(self, word: str) -> List[int]:
        out = []
        w = [self._b2u[b] for b in word.encode("utf-8")]
        while len(w) > 1:
            best, bi = None, -1
            for i in range(len(w) - 1):
                r = self.bpe_ranks.get((w[i], w[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            w = w[:bi] + [w[bi] + w[bi + 1]] + w[bi + 2:]
        for piece in w:
            pid = self.piece_to_id.get(piece)
            if pid is None:
                out.extend(self.piece_to_id.get(c, self.unk_id) for c in piece)
            else:
                out.append(pid)
        return out

    # ------------------------------------------------------------ detokenize
    def token_to_piece(self, tok: int, special: bool = False) -> bytes:
        if tok < 0 or tok >= self.n_vocab:
            return b""
        t, ty = self.tokens[tok], self.types[tok]
        if ty in (TOKEN_CONTROL, TOKEN_UNUSED) or ty == TOKEN_UNKNOWN:
            return t.encode() if (special and ty == TOKEN_CONTROL) else b""
        if self.model == "gpt2":
            return bytes(self._u2b.get(c, ord("?")) for c in t) if ty != TOKEN_USER else t.encode()
        if ty == TOKEN_BYTE:
            return bytes([int(t[3:5], 16)])
        return t.replace(SPACE, " ").encode("utf-8")

    def detokenize(self, tokens: Sequence[int], prev_tokens: Optional[Sequence[int]] = None,
                   special: bool = False) -> bytes:
        out = b"".join(self.token_to_piece(int(t), special) for t in tokens)
        # llama.cpp strips the SPM space prefix of the first piece after BOS when decoding from the start
        if self.model == "llama" and self.add_space_prefix and not prev_tokens and out.startswith(b" "):
            first_real = next((int(t) for t in tokens if self.types[int(t)] not in (TOKEN_CONTROL,)), None)
            if first_real is not None:
                out = out[1:]
        return out

    def is_eog(self, tok: int) -> bool:
        return tok == self.eos_id or (self.eot_id is not None and tok == self.eot_id)
