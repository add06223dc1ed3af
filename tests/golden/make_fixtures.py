#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the reference's own test data.

Run once in the build container (it reads /root/reference, which does not exist on
the GPU box); the outputs are committed so tests never read the reference at run time.

Inputs (data files the reference's tests hold; no reference source is copied):
  * RoaringBitmap/src/test/resources/testdata/{bitmapwithruns,bitmapwithoutruns,
    crashproneinput1..8}.bin  -> copied byte-for-byte to tests/golden/testdata/
    (used by RBT/TestAdversarialInputs.java:32-55)
  * real-roaring-dataset/src/main/resources/real-roaring-dataset/<name>.zip
    -> tests/golden/realdata/<name>.npz : the 200 integer sets in zip-entry order
    (ZipRealDataRetriever.fetchBitPositions, real-roaring-dataset/src/main/java/
    org/roaringbitmap/ZipRealDataRetriever.java:40-69), stored as one concatenated
    uint32 `values` array plus `offsets` (len 201).
  * RoaringBitmap/src/test/resources/testdata/ornot-fuzz-failure.json (the two base64 bitmaps of
    RBT/TestRoaringBitmapOrNot.java:376-424 testBigOrNot / testBigOrNotStatic)
    -> tests/golden/testdata/ornot_fuzz_{l,r}.bin.gz, the decoded serialized bytes, gzipped
  * RoaringBitmap/src/test/resources/testdata/{testIssue260,offset_failure_case_1..3}.txt (the
    comma-separated value lists of RBT/TestConcatenation.java:32-37, addOffset's cases)
    -> tests/golden/testdata/addoffset_<name>.u32.gz, the values as little-endian uint32, gzipped
  * The known-answer constants of jmh/src/test/java/org/roaringbitmap/realdata/
    RealDataBenchmark{Or,And,AndNot,Xor,WideOrNaive,WideAndNaive}Test.java are
    transcribed (as numbers) into known_answers.json.
"""
import base64
import gzip
import json
import os
import shutil
import zipfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
TESTDATA_SRC = os.path.join(REF, "RoaringBitmap/src/test/resources/testdata")
REALDATA_SRC = os.path.join(REF, "real-roaring-dataset/src/main/resources/real-roaring-dataset")
DATASETS = ["census1881", "census1881_srt", "uscensus2000", "wikileaks-noquotes",
            "wikileaks-noquotes_srt"]

# Transcribed from jmh/src/test/java/org/roaringbitmap/realdata/*Test.java
# (pairwise sums over k = 0..198 of |b[k] op b[k+1]|; wide ops over all 200).
KNOWN_ANSWERS = {
    "census1881": {"or": 2007691, "or_nocard": 192344014, "and": 23, "xor": 2007668,
                   "andnot": 1003836, "wide_or": 988653, "wide_and": 0},
    "census1881_srt": {"or": 1360167, "or_nocard": 113309680, "and": 206, "xor": 1359961,
                       "andnot": 679375, "wide_or": 656346, "wide_and": 0},
    "uscensus2000": {"or": 11954, "or_nocard": 1085687199, "and": 0, "xor": 11954,
                     "andnot": 5970, "wide_or": 5985, "wide_and": 0},
    "wikileaks-noquotes": {"or": 541893, "or_nocard": 43309741, "and": 3327, "xor": 538566,
                           "andnot": 271605, "wide_or": 242540, "wide_and": 0},
    "wikileaks-noquotes_srt": {"or": 574463, "or_nocard": 28702307, "and": 152, "xor": 574311,
                               "andnot": 286904, "wide_or": 236436, "wide_and": 0},
}
KNOWN_SOURCES = {
    "or": "RealDataBenchmarkOrTest.java EXPECTED_RESULTS",
    "or_nocard": "RealDataBenchmarkOrTest.java EXPECTED_RESULTS_NO_CARDINALITY",
    "and": "RealDataBenchmarkAndTest.java",
    "xor": "RealDataBenchmarkXorTest.java",
    "andnot": "RealDataBenchmarkAndNotTest.java",
    "wide_or": "RealDataBenchmarkWideOrNaiveTest.java",
    "wide_and": "RealDataBenchmarkWideAndNaiveTest.java (asserts 0)",
}


def main():
    td = os.path.join(HERE, "testdata")
    os.makedirs(td, exist_ok=True)
    names = ["bitmapwithruns.bin", "bitmapwithoutruns.bin"] + [
        f"crashproneinput{i}.bin" for i in range(1, 9)]
    for n in names:
        shutil.copyfile(os.path.join(TESTDATA_SRC, n), os.path.join(td, n))

    with open(os.path.join(TESTDATA_SRC, "ornot-fuzz-failure.json")) as f:
        bms = json.load(f)["bitmaps"]
    for tag, b in zip("lr", bms[:2]):
        with gzip.GzipFile(os.path.join(td, f"ornot_fuzz_{tag}.bin.gz"), "wb", mtime=0) as g:
            g.write(base64.b64decode(b))

    for n in ("testIssue260", "offset_failure_case_1", "offset_failure_case_2", "offset_failure_case_3"):
        with open(os.path.join(TESTDATA_SRC, n + ".txt")) as f:
            vals = np.array([int(x) for x in f.readline().strip().split(",")], dtype="<u4")
        with gzip.GzipFile(os.path.join(td, f"addoffset_{n}.u32.gz"), "wb", mtime=0) as g:
            g.write(vals.tobytes())

    rd = os.path.join(HERE, "realdata")
    os.makedirs(rd, exist_ok=True)
    for ds in DATASETS:
        z = zipfile.ZipFile(os.path.join(REALDATA_SRC, ds + ".zip"))
        # ZipInputStream walks local headers in file order
        infos = sorted(z.infolist(), key=lambda i: i.header_offset)
        sets = []
        for info in infos:
            line = z.read(info).decode().splitlines()[0]
            sets.append(np.array([int(x) for x in line.split(",")], dtype=np.uint32))
        offsets = np.zeros(len(sets) + 1, dtype=np.int64)
        offsets[1:] = np.cumsum([len(s) for s in sets])
        np.savez_compressed(os.path.join(rd, ds + ".npz"), values=np.concatenate(sets),
                            offsets=offsets)
        print(ds, len(sets), int(offsets[-1]))

    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump({"values": KNOWN_ANSWERS, "sources": KNOWN_SOURCES}, f, indent=1)


if __name__ == "__main__":
    main()
