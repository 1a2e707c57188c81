# Drop-in mirror of the reference's `models` package (QasimKhan5x/dgcnn.pytorch):
# same module paths and public names, backed by the dgx HIP engine.
