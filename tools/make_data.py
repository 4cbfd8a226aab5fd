"""Generate the synthetic datasets the CLIs and run.sh read.

The reference trains on the Amazon fine-food-reviews CSVs (S3 links in its
README.md:348-350, absent here), so:

  dense  (default): ./data/train.csv + ./data/test.csv in the reference schema
         (header "0".."1023","Score"; 1024 hashed L2-normalised features, labels
         1..5, ~90k train / 4,877 test rows), calibrated so that full-batch LR
         reaches ~0.47 test accuracy (the reference's offline ground truth);
  sparse: ./data/train.svm + ./data/test.svm (LIBSVM) with --features hashed
         sparse features (BASELINE.json configs 4/5; --binary for labels 0/1).

Usage: python tools/make_data.py [--out ./data] [--sparse] [--rows N] [--test-rows T]
                                 [--features F] [--binary] [--seed S]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="./data")
    ap.add_argument("--sparse", action="store_true")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--test-rows", type=int, default=None)
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--binary", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    from psx.utils.data import FINEFOOD_TEST_ROWS, save_libsvm, synth_finefood, synth_sparse, write_csv

    os.makedirs(a.out, exist_ok=True)
    if a.sparse:
        F = a.features or (1 << 20)
        kw = dict(num_features=F, labels="binary" if a.binary else "finefood")
        tr = synth_sparse(a.rows or 1_000_000, seed=a.seed, **kw)
        te = synth_sparse(a.test_rows or 20000, seed=a.seed + 1, **kw)
        save_libsvm(tr, os.path.join(a.out, "train.svm"))
        save_libsvm(te, os.path.join(a.out, "test.svm"))
        print(f"wrote {a.out}/train.svm ({tr.rows} rows, {tr.nnz} nnz) and test.svm ({te.rows} rows), F={F}")
        return
    F = a.features or 1024
    tr = synth_finefood(a.rows or 90000, num_features=F, seed=a.seed)
    te = synth_finefood(a.test_rows or FINEFOOD_TEST_ROWS, num_features=F, seed=a.seed + 1)
    write_csv(tr, os.path.join(a.out, "train.csv"))
    write_csv(te, os.path.join(a.out, "test.csv"))
    print(f"wrote {a.out}/train.csv ({tr.rows} rows) and test.csv ({te.rows} rows), F={F}")


if __name__ == "__main__":
    main()
