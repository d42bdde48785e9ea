"""Reference package path ``AlphaGo.preprocessing`` (featurizer + SGF->HDF5 converter)."""
