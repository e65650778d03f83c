"""``src.download_data``: fetch the paper's dataset (needs ``gdown`` and network)."""
from deeplearninginassetpricing_paperreplication_amd.data.download import (  # noqa: F401
    DATASETS_ZIP_ID, EXPECTED_SIZES, GDRIVE_FOLDER_ID, check_data_exists, download_all_data,
    download_datasets_zip, download_from_folder, main, print_data_info)

if __name__ == "__main__":
    main()
