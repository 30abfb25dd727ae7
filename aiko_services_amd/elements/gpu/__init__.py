"""GPU-resident elements (MI355X): synthetic decode, preprocess, ResNet-50, top-k."""
