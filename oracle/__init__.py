"""TEST INFRASTRUCTURE ONLY — the parity oracle for the HMM hot path.

Nothing in this package is part of the product.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import it, and only as the checker (or, for the
baseline, as the thing timed on the host cores).  The product path
(pytorch_hmm_amd) never imports, links or executes anything under oracle/.

Contents
  hmm_oracle.py  CPU restatement of the reference algorithms in torch-CPU ops, in the
                 reference's exact op order, so its outputs are bit-identical to the
                 reference on the same machine (pinned by tests/golden/*.npz, which were
                 produced by running the reference itself: tests/golden/make_golden.py).
  hmm_oracle.c   Plain-C restatement of the integer/exact parts (max-plus Viterbi with
                 first-index ties, HSMM segment Viterbi with torch's strided-sum order)
                 and float64 forward-backward / emission references for tolerance checks.
                 Built into oracle/lib/liboracle.so by oracle/Makefile.
"""
