"""FASTA / FASTQ files (drop-in for src/data_file.py): extension check, plain or
gzip text, parsed into the containers of records.py."""

from __future__ import annotations

import gzip
import pickle
from typing import Optional, Set

from records import FASTAQRecordContainer, FASTARecordContainer, NoRecordsInData, RecordContainer


class InvalidExtensionError(Exception):
    def __init__(self, message: str = "") -> None:
        super().__init__(message)


class NoRecordsInDataFile(Exception):
    def __init__(self, message: str = "") -> None:
        super().__init__(message)


class DataFile:
    """Base: subclasses set EXTENSIONS and the container type."""

    EXTENSIONS: Optional[Set[str]] = None

    def __init__(self, file_path: str) -> None:
        if not self.EXTENSIONS:
            raise NotImplementedError("EXTENSIONS must be defined.")
        if not any(file_path.endswith(ext) for ext in self.EXTENSIONS):
            raise InvalidExtensionError(f"Invalid file extension. Expected one of {self.EXTENSIONS}, got {file_path}")
        self.container: RecordContainer = self.get_container_type()
        self.parse_file(file_path)

    def get_container_type(self) -> RecordContainer:
        raise NotImplementedError("This method must be implemented in subclasses.")

    def parse_file(self, file_path: str) -> None:
        try:
            self.container.parse_records(self.load_file(file_path))
        except NoRecordsInData:
            raise NoRecordsInDataFile(f"No valid records found in file: {file_path}")

    def load_file(self, file_path: str) -> str:
        opener = gzip.open if file_path.endswith(".gz") else open
        with opener(file_path, "rt", encoding="utf-8") as f:
            return f.read()

    def dump(self, output_file: str) -> None:
        with open(output_file, "wb") as f:
            pickle.dump(self.container, f)


class FASTAFile(DataFile):
    EXTENSIONS = {".fa", ".fa.gz"}

    def get_container_type(self) -> FASTARecordContainer:
        return FASTARecordContainer()


class FASTAQFile(DataFile):
    EXTENSIONS = {".fq", ".fq.gz"}

    def get_container_type(self) -> FASTAQRecordContainer:
        return FASTAQRecordContainer()
