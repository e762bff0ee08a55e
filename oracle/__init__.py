"""CPU oracle for the semantic loop-closure gate -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, what the reference
(wadewilliamsw1234/Multi-level-Indoor-SLAM, ``scripts/semantic_gating``) computes on
the hot path.  It exists to *check* the HIP product path, never to stand in for it:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it.  The product package (``mlgate``) never imports it and
fails loudly when its HIP library is missing.

Pinning (see DESIGN.md "Oracle"):
  * retrieval / gate / IMU floor labels / cross-correlation -- pinned against
    golden vectors captured by importing the reference in the build container
    (``tests/golden/make_goldens.py``) and against the gate counts published in
    ``results/semantic_gating/*.txt``.
  * ViT-B/14 descriptor path -- the weights come from torch.hub and cannot be
    fetched offline, so the restatement is pinned architecturally against
    ``transformers.Dinov2Model`` (same network, seeded weights, 518x518 where the
    hub pos-embed interpolation is the identity).  Descriptor values themselves are
    "parity unpinned" against the real reference weights.
  * cv2.resize INTER_LINEAR (uint8) -- OpenCV is absent; restated from its
    published fixed-point algorithm, "parity unpinned".
"""
