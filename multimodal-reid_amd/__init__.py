"""multimodal_reid_amd — MI355X-native CLIP-ReID inference + retrieval path."""
