"""WordCount over text:// LineRecord tables: LocalDebug oracle vs the process executor, and the
@device_function tokeniser's host path (the GPU path is in test_gpu_text.py)."""
import os
from collections import Counter

import dryad_amd as D
from dryad_amd.models.wordcount import synthetic_corpus, word_count_query


def test_text_provider_partitions_cut_at_newlines(tmp_path):
    p = str(tmp_path / "t.txt")
    with open(p, "w") as f:
        f.write("a b\r\nc d e\n\nlast")
    from dryad_amd.io.providers import provider_for
    uri = f"text://{p}?partitions=3"
    prov = provider_for(uri)
    parts = [prov.read_partition(uri, i, None) for i in range(prov.stream_info(uri)[0])]
    assert [r.Line for part in parts for r in part] == ["a b", "c d e", "", "last"]


def test_wordcount_executor_matches_oracle_and_counter(tmp_path):
    p = synthetic_corpus(str(tmp_path / "corpus.txt"), 3000, vocab=500)
    uri = f"text://{p}?partitions=4"
    ld = D.DryadLinqContext(1)
    ld.LocalDebug = True
    a = dict(word_count_query(ld, uri))
    b = dict(word_count_query(D.DryadLinqContext(2), uri))
    with open(p) as f:
        exp = Counter(f.read().split())
    assert a == dict(exp) and b == dict(exp)


def test_wordcount_to_text_store(tmp_path):
    p = synthetic_corpus(str(tmp_path / "c.txt"), 200, vocab=50)
    out = str(tmp_path / "out")
    c = D.DryadLinqContext(2)
    word_count_query(c, f"text://{p}?partitions=2").Select(lambda t: f"{t[0]}\t{t[1]}").ToStore(
        f"text://{out}").SubmitAndWait()
    got = {}
    for fn in os.listdir(out):
        with open(os.path.join(out, fn)) as f:
            for line in f:
                w, n = line.rstrip("\n").split("\t")
                got[w] = int(n)
    with open(p) as f:
        assert got == dict(Counter(f.read().split()))
