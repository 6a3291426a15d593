"""CPU oracle for the MS-UNet / Swin training hot path -- TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``semantic_segmentation_of_stylegan2_artifacts_amd``) never imports
anything from here and fails loudly when its HIP library is missing.

Contents (plain PyTorch fp32 on the CPU, functional, no nn.Module state):

* ``swin_block``   -- restatement of torchvision v1 ``SwinTransformerBlock`` /
  ``shifted_window_attention`` (third-party, absent from the reference tree; version
  unpinned by the reference).  Parity of this piece is *unpinned* by any reference
  artefact: the reference only pins its parameter layout
  (``network/pretrained_weights/structure_of_MSUNet.txt``).
* ``msunet``       -- functional restatement of ``network/model_parts.py::MSUNetSys``
  (topology pinned by golden vectors produced by importing the reference module,
  see ``tests/golden/gen_golden.py``).
* ``dynamic_loss`` -- restatement of ``loss/DynamicLoss.py`` (pinned by golden vectors
  produced by importing the reference module directly).
* ``metrics``      -- restatement of ``scripts/validation_functions.py`` soft/binary
  metric formulas.
"""
