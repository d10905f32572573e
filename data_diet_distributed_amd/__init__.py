"""MI355X-native Data Diet scoring and pruning (drop-in for the scoring path of
TejasPote/data_diet_distributed).

  get_scores_and_prune.sparse_loader   reference-signature entry point
  scoring.ScoringEngine                 K-checkpoint EL2N + GraNd, sharded, global select
  resnet                                state_dict-compatible ResNet-18/34/50/101/152
  loader / checkpoints / subset_index   data feed, checkpoint formats, keep-set artefact
  _capi                                 ctypes binding of libdd.so (include/dd_capi.h)
"""
__all__ = ["get_scores_and_prune", "scoring", "resnet", "loader", "checkpoints",
           "subset_index", "synthetic", "config"]
