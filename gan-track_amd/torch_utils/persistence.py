"""Snapshot plumbing.  The reference embeds class source into pickles
(SG3/torch_utils/persistence.py:35-130); this build keeps plain module classes and saves
state_dict-based snapshots (training_loop_mi_multimodal.save_snapshot).  `persistent_class` is a
no-op decorator kept for API compatibility."""


def persistent_class(orig_class):
    return orig_class


def is_persistent(obj):
    return False
