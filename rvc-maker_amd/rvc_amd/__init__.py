"""rvc_amd -- MI355X-native RVC voice-conversion hot path (host side).

Python host mirroring the reference interfaces (VC.pipeline, Synthesizer.infer,
HubertModel.extract_features, RMVPE.infer_from_audio) over the C-ABI library
librvc_amd.so (include/rvc_amd.h).  There is no CPU fallback.
"""
