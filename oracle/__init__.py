"""CPU oracle for the FiBiNET training path -- TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithm (YOUNESELBOUKNIFY/Ctr_recommendation,
``src/model_fibinet.py`` + the per-step part of ``src/train_fibinet.py``) with stock
PyTorch CPU ops, and the data path (``src/dataloader.py``, ``src/Prediction.py``'s collator and
export) with pandas / numpy (``oracle/collate_ref.py``).  It exists to *check* the HIP path, never to run it:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
  may import it;
* nothing in ``ctr_recommendation_amd/`` imports it (``tests/test_lib.py::
  test_product_never_imports_oracle`` enforces this).

Pinning (see DESIGN.md "Oracle"): the reference ships no tests or fixtures and running it
was denied in the survey container, so the oracle is pinned by

1. the one known-answer value recorded before that denial (seed 0, d=16,
   train mode, first four probabilities ``[0.3714, 0.4710, 0.4549, 0.6018]``);
2. the App. B state_dict contract and parameter counts (2 095 726 at d=16);
3. the 160-point OneCycleLR trace logged in ``Notebooks/train_predict_kaggle.ipynb``
   (fixture ``tests/golden/kaggle_lr_trace.json``).
"""
