"""Import-path shim: `from simple_knn._C import distCUDA2` resolves to the MI355X implementation."""
