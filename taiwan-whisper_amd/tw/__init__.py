"""tw — MI355X-native Whisper distillation engine (drop-in for the taiwan-whisper hot path).

Host side mirrors the reference's interfaces (training/run_distillation.py train_step,
training/create_student_model.py, HF WhisperForConditionalGeneration / WhisperFeatureExtractor
attributes the reference touches); all arithmetic runs in libtw_hip.so (gfx950 HIP kernels).
"""
__version__ = "0.1.0"
