"""``src.generate_synthetic_data``: reference-compatible synthetic panels (same seed -> same files)."""
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import (  # noqa: F401
    apply_missing_values, create_individual_npz, create_macro_npz, generate_all_splits,
    generate_characteristics, generate_dataset, generate_factor_loadings, generate_factor_returns,
    generate_macro_features, generate_missing_pattern, generate_returns, main)

if __name__ == "__main__":
    main()
