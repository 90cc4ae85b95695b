"""xspect2_amd — MI355X-native k-mer x filter probe path for XspecT.

Host side in Python (the reference's model surface), hot path in hand-written
gfx950 HIP behind the C ABI of ``include/xspect_hip.h`` (libxspect_hip.so).

Submodules mirror the reference modules they replace:
  probabilistic_filter_model         <- xspect.models.probabilistic_filter_model
  probabilistic_filter_svm_model     <- xspect.models.probabilistic_filter_svm_model
  probabilistic_single_filter_model  <- xspect.models.probabilistic_single_filter_model
  probabilistic_filter_mlst_model    <- xspect.models.probabilistic_filter_mlst_model
  result                             <- xspect.models.result / mlst_result
  classify                           <- xspect.classify
"""
__version__ = "0.1.0"
