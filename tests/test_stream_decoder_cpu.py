"""Incremental detokenization for the SSE streams (``dgi.utils.tokenizer.StreamDecoder``): the
pieces concatenate to the full decode, a character split over tokens is emitted once complete
(no U+FFFD in the stream), and word-boundary spaces survive (decoding each token alone drops them)."""
import random

from dgi.utils.tokenizer import ByteTokenizer, StreamDecoder


def _stream(tok, ids):
    d = StreamDecoder(tok)
    pieces = [d.add(i) for i in ids]
    return pieces, "".join(pieces) + d.flush()


def test_utf8_split_over_byte_tokens_and_unknown_ids():
    t = ByteTokenizer(vocab_size=128256)
    s = "héllo wörld — 漢字 ok"
    ids = t.encode(s, add_bos=False) + [300, 5000] + t.encode(" end", add_bos=False)
    pieces, out = _stream(t, ids)
    assert out == t.decode(ids) == s + "□□ end"
    assert not any("�" in p for p in pieces)
    # every unknown id is visible at once (SSE TTFT of a random-init model = its first token)
    assert _stream(t, [4000])[0] == ["□"]


def test_random_sequences_concatenate_to_the_full_decode():
    t = ByteTokenizer(vocab_size=512)
    rng = random.Random(0)
    for _ in range(200):
        ids = [rng.randrange(0, 512) for _ in range(rng.randrange(1, 40))]
        assert _stream(t, ids)[1] == t.decode(ids)


class _SentencePieceLike:
    """Word pieces with a '▁' word-boundary marker; decode strips the leading space of the text
    (SentencePiece), so decoding tokens one by one loses every space."""
    vocab = ["▁the", "▁quick", "▁br", "own", "▁fox", "!", "▁é", "t", "é"]

    def decode(self, ids, skip_special_tokens=True):
        return "".join(self.vocab[i] for i in ids).replace("▁", " ").lstrip(" ")


def test_word_boundary_spaces_survive():
    t = _SentencePieceLike()
    ids = [0, 1, 2, 3, 4, 5, 6, 7, 8]
    pieces, out = _stream(t, ids)
    assert out == t.decode(ids) == "the quick brown fox! été"
    assert "".join(t.decode([i]) for i in ids) != out          # what per-token decoding produced
