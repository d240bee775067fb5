"""ORACLE -- TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's GE2E training hot path
(hwidong-na/PyTorch_Speaker_Verification), used to CHECK the HIP product path.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything from here, and only as the checker / the timed CPU baseline --
never as the thing measured or shipped.  The product package
``pytorch_speaker_verification_amd`` never imports this package.

Modules
  ge2e_np     numpy fp64 restatement of utils.py:27-132 + speech_embedder_net.py:35-49
              (forward and closed-form backward).
  lstm_np     numpy fp64 restatement of the SpeechEmbedder forward
              (speech_embedder_net.py:27-33: nn.LSTM, last frame, Linear, L2 norm),
              its BPTT backward, and clip_grad_norm_ + SGD (train_speech_embedder.py:63-65).
  torch_port  the same path as a PyTorch-CPU port (nn.LSTM on oneDNN, the reference's
              CPU execution path) -- the bench's cpu_baseline and the full-size checker.

Pinning: ge2e_np and lstm_np are checked in tests/test_oracle_golden.py against the
golden vectors in tests/golden/, which tests/golden/make_golden.py produced by running
the reference itself (imported read-only in the build container), including the
reference's own utils.py:166-173 example (KAT-0) and its *_prior loop twins.
"""
