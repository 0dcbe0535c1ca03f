"""GGUF-metadata tokenizer (llama-p2p_amd/tokenizer.py) against independent
implementations, offline: a SentencePiece BPE model trained here with `sentencepiece` (the LLaMA /
TinyLlama "llama" tokenizer family: identity normaliser, dummy prefix, byte fallback -- what
llama.cpp's llm_tokenizer_spm expects) and a byte-level BPE trained with `tokenizers` using the
Llama-3 pre-tokenizer regex (the "gpt2" / "llama-bpe" family).  Parity: identical token ids and
exact detokenize round trips.  No reference model file exists offline, so the vocabularies are
small trained ones; the algorithms compared are the same."""
import json
import random

import pytest

from llama_p2p_amd.tokenizer import (LLAMA3_PRETOKENIZE, TOKEN_BYTE, TOKEN_CONTROL, TOKEN_NORMAL,
                                     TOKEN_UNKNOWN, Tokenizer)

WORDS = ("the quick brown fox jumps over lazy dog hello world llama peer network inference model cache "
         "gossip token secret key prompt result distributed node request 2024 3.14 don't it's").split()
TEXTS = ["hello world", "the llama jumps over the lazy peer", "  two  spaces  ", "numbers 12345 and 3.14159",
         "Ünïcödé çàfé naïve", "tabs\tand\nnewlines\n\nhere", "don't stop, it's a gossip-network!",
         "emoji 🦙 and 中文字符", "x", "punctuation ?!.,;:()[]{}<>"]


def _corpus(path, n=3000):
    r = random.Random(0)
    lines = [" ".join(r.choice(WORDS) for _ in range(r.randint(4, 14))) for _ in range(n)]
    lines += TEXTS[:7]
    path.write_text("\n".join(lines), encoding="utf-8")
    return str(path)


def test_spm_matches_sentencepiece(tmp_path):
    spm = pytest.importorskip("sentencepiece")
    corpus = _corpus(tmp_path / "c.txt")
    prefix = str(tmp_path / "spm")
    spm.SentencePieceTrainer.train(input=corpus, model_prefix=prefix, vocab_size=320, model_type="bpe",
                                   byte_fallback=True, character_coverage=1.0, normalization_rule_name="identity",
                                   remove_extra_whitespaces=False, add_dummy_prefix=True, minloglevel=2)
    sp = spm.SentencePieceProcessor(model_file=prefix + ".model")
    n = sp.get_piece_size()
    types = [TOKEN_UNKNOWN if sp.is_unknown(i) else TOKEN_CONTROL if sp.is_control(i)
             else TOKEN_BYTE if sp.is_byte(i) else TOKEN_NORMAL for i in range(n)]
    tok = Tokenizer([sp.id_to_piece(i) for i in range(n)], [sp.get_score(i) for i in range(n)], types, "llama",
                    bos_id=sp.bos_id(), eos_id=sp.eos_id(), unk_id=sp.unk_id())
    for s in TEXTS:
        ours = tok.tokenize(s.encode(), add_bos=False)
        assert ours == sp.encode(s), s
        assert tok.tokenize(s.encode(), add_bos=True) == [sp.bos_id()] + ours
        assert tok.detokenize(ours).decode("utf-8") == s, s


def test_bpe_matches_tokenizers(tmp_path):
    tk = pytest.importorskip("tokenizers")
    from tokenizers import Regex, decoders, models, pre_tokenizers, trainers

    t = tk.Tokenizer(models.BPE())
    t.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_PRETOKENIZE), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    t.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=600, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                             show_progress=False)
    t.train([_corpus(tmp_path / "c.txt")], tr)
    spec = json.loads(t.to_str())
    vocab = spec["model"]["vocab"]
    merges = [m if isinstance(m, str) else " ".join(m) for m in spec["model"]["merges"]]
    tokens = [None] * len(vocab)
    for piece, i in vocab.items():
        tokens[i] = piece
    tok = Tokenizer(tokens, model="gpt2", merges=merges, add_bos=False, add_space_prefix=False)
    for s in TEXTS:
        ours = tok.tokenize(s.encode(), add_bos=False)
        assert ours == t.encode(s).ids, s
        assert tok.detokenize(ours).decode("utf-8") == s, s


def test_spm_segment_cache_is_exact():
    """Segmenting SPM text before every SPACE that follows a non-SPACE (the per-segment cache) gives
    the same ids as merging the whole text, for a vocabulary with no piece holding such a pair; a
    vocabulary that holds one falls back to whole-text merging."""
    from llama_p2p_amd import gguf
    from llama_p2p_amd.tokenizer import SPACE, Tokenizer

    toks, scores, types = gguf.synthetic_spm_vocab(4096)
    tok = Tokenizer(toks, scores, types, "llama", bos_id=1, eos_id=2)
    assert tok._spm_split
    rng = random.Random(5)
    words = ["node", "peer", "the", "llama", "a", "12", "x.y", "é", "  ", "   "]
    for _ in range(50):
        s = " ".join(rng.choice(words) for _ in range(rng.randint(1, 40)))
        whole = tok._spm_seg((" " + s).replace(" ", SPACE))
        assert tok.tokenize(s.encode(), add_bos=False) == whole
    bad = Tokenizer(list(toks) + ["e" + SPACE], list(scores) + [0.0], list(types) + [TOKEN_NORMAL], "llama")
    assert not bad._spm_split
