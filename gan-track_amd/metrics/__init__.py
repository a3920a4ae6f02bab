"""Quality metrics of the training loop: FID-50k per modality (SG3/metrics/*_mi_multimodal.py)."""
