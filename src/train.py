"""``src.train``: ``python -m src.train --data_dir D [...]`` (reference CLI + --device/--precision)."""
from deeplearninginassetpricing_paperreplication_amd.train.cli import main  # noqa: F401
from deeplearninginassetpricing_paperreplication_amd.train.metrics import (  # noqa: F401
    compute_max_drawdown, compute_sharpe)
from deeplearninginassetpricing_paperreplication_amd.train.trainer import (  # noqa: F401
    evaluate, train_3phase, train_epoch)

if __name__ == "__main__":
    main()
