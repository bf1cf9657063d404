"""CPU oracle for the autoencoder-CF hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in the product package (`omnidirectional_collaborative_filtering_amd`) imports,
links or executes anything under `oracle/`.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg use it, and only as the checker / the timed CPU baseline.

Modules
-------
batch_oracle   NumPy/pure-Python restatement of `data_reader.py` (build_sparse_batch,
               build_sparse_batch_fixed_split, data_gen) including the exact NumPy legacy
               RandomState draw sequence.  PINNED against the reference itself: the golden
               fixtures in tests/golden/ were produced by importing /root/reference/data_reader.py
               (script: tests/golden/make_golden.py) and this restatement reproduces them bit for bit.
model_oracle   NumPy float64/float32 restatement of the Keras 2.0.4 / TF 1.3 arithmetic the
               reference delegates to (Dense, sigmoid/tanh, Dropout, multiply-mask, MSE,
               Adagrad/RMSprop/Adam, the train.py metrics and compute_full_RMSE).
               PARITY UNPINNED: TF/Keras are absent from this image and the reference has no
               tests or fixtures for the model path, so this restatement is pinned only by the
               published Keras 2.0.4 equations it cites (see DESIGN.md "Oracle").
"""
