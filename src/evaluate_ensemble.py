"""``src.evaluate_ensemble``: ``python -m src.evaluate_ensemble --data_dir D --checkpoint_dirs ...``."""
from deeplearninginassetpricing_paperreplication_amd.analysis.ensemble import (  # noqa: F401
    compute_sharpe, evaluate_ensemble, get_weights_from_model, load_model, main)

if __name__ == "__main__":
    main()
