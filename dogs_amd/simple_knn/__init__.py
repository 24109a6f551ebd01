"""Drop-in `simple_knn` (reference submodules/simple-knn) on MI355X: `from simple_knn._C import distCUDA2`."""
