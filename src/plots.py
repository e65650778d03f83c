"""``src.plots``: ``python -m src.plots --data_dir D --checkpoint_dirs ... [--output_dir]``."""
from deeplearninginassetpricing_paperreplication_amd.analysis.ensemble import load_model  # noqa: F401
from deeplearninginassetpricing_paperreplication_amd.analysis.plots import (  # noqa: F401
    generate_all_plots, get_date_range, main, plot_cumulative_sdf, plot_monthly_returns,
    plot_sharpe_comparison, plot_summary_statistics, plot_training_curves)

if __name__ == "__main__":
    main()
