"""Device text kernels (line split, tokenise, hashed word count) vs Python string ops."""
from collections import Counter

import pytest
import torch

pytestmark = pytest.mark.gpu


def _heap(s: bytes):
    return torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()


@pytest.mark.parametrize("text", [b"a b\r\nc  d\te\n\nlast", b"one\n", b"   \n\n", b"x", b"", b"mac\rlines\r\rend\r"])
def test_lines_and_tokens_match_python(text):
    from dryad_amd.ops import text as TX
    h = _heap(text) if text else torch.zeros(0, dtype=torch.uint8, device="cuda")
    off, ln = TX.lines(h)
    import re
    exp_lines = re.split(rb"\r\n|\r|\n", text)
    if exp_lines and exp_lines[-1] == b"":
        exp_lines.pop()
    got = [text[o:o + n] for o, n in zip(off.tolist(), ln.tolist())]
    assert got == exp_lines
    to, tl = TX.tokens(h)
    assert [text[o:o + n] for o, n in zip(to.tolist(), tl.tolist())] == text.split()


def test_word_count_matches_counter(tmp_path):
    from dryad_amd.models.wordcount import synthetic_corpus
    from dryad_amd.ops import text as TX
    p = synthetic_corpus(str(tmp_path / "c.txt"), 20000, vocab=3000)
    data = open(p, "rb").read()
    got = dict(TX.word_count(_heap(data)))
    assert got == dict(Counter(data.decode().split()))


def test_word_count_table_matches_counter(tmp_path):
    """(word, count) groups built as an HBM table (device-compacted word heap, Int32 counts)."""
    from dryad_amd.models.wordcount import synthetic_corpus
    from dryad_amd.ops import text as TX
    p = synthetic_corpus(str(tmp_path / "c.txt"), 20000, vocab=3000)
    data = open(p, "rb").read()
    t = TX.word_count_table(_heap(data))
    assert t is not None and t.strs["Item1"].is_cuda and t.cols["Item2"].dtype == torch.int32
    got = dict(t.to_objects())
    assert got == dict(Counter(data.decode().split()))
    assert TX.word_count_table(_heap(b"   \n")) is None


def test_wordcount_query_on_gpu_executor(tmp_path):
    import dryad_amd as D
    from dryad_amd.models.wordcount import synthetic_corpus, word_count_query
    p = synthetic_corpus(str(tmp_path / "c.txt"), 5000, vocab=800)
    uri = f"text://{p}?partitions=2"
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = 2
    got = dict(word_count_query(g, uri))
    with open(p) as f:
        assert got == dict(Counter(f.read().split()))
    fb = {op for _, op, _ in g._get_executor().last_result["fallbacks"]}
    assert "read" not in fb and "apply" not in fb
